"""BERT encoder + sequence-classification head on the gfx950 kernels.

BASELINE.json config 5 is "BERT-base fine-tune, synthetic GLUE, DP" (SURVEY.md
section 2.7 K13: LayerNorm, GELU, embedding, attention; not present in the
reference, which only names Keras workloads).  The architecture is the
standard post-LN BERT (``hidden 768, 12 layers, 12 heads, FFN 3072, GELU(erf),
LN eps 1e-12, dropout 0.1``) with a tanh pooler over [CLS] and a linear
classifier, randomly initialised (N(0, 0.02), as BERT does).

MI355X execution (bf16 CUDA tensors, native ops):

* one autograd node per encoder layer (:class:`_LayerFn`), hand-scheduled:
    qkv  = x Wqkv^T + b            (one N=2304 GEMM, bias in the epilogue)
    ctx  = attention(qkv)          (fused flash-style kernel, reads qkv in place)
    y1   = LN(x + drop(ctx Wo^T + bo))        (residual + dropout fused into LN)
    f    = GELU(y1 W1^T + b1)      (bias + GELU in the epilogue, pre-act kept)
    y2   = LN(y1 + drop(f W2^T + b2))
  backward: GELU' fused into the W2-dgrad epilogue, the residual gradient
  summed into the W1/Wqkv dgrad epilogues (beta = 1), weight gradients split-K
  straight into the flat gradient arena, bias gradients by column-sum kernels,
  LN dgamma/dbeta accumulated into the arena, DDP notified per parameter;
* embeddings: gather-sum kernel + LN(+dropout); fp32 tables whose gradients
  are scattered with hardware fp32 atomics into the arena;
* key-padding mask given per sequence as a valid length (``attention_mask``
  must be a prefix mask, as produced by BERT tokenizers with right padding).

CPU tensors (tests) run the same math in plain PyTorch (:meth:`_torch_forward`),
which is also the fp32 numerics reference for the GPU tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import config
from ..ops import _ext, raw
from ..ops.dropout import next_seed
from ..runtime import side_stream
from ..runtime.side_stream import SideWork


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    num_labels: int = 2
    pad_token_id: int = 0

    @classmethod
    def base(cls, **kw):
        return cls(**kw)

    @classmethod
    def large(cls, **kw):
        d = dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096)
        d.update(kw)
        return cls(**d)

    @classmethod
    def tiny(cls, **kw):
        d = dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                 max_position_embeddings=128)
        d.update(kw)
        return cls(**d)


def _grad_out(p):
    """(sink, owned): the arena gradient slice if resident, else a fresh zero buffer to return."""
    g = getattr(p, "grad", None)
    if g is not None and getattr(p, "_ca_arena", False) and g.is_contiguous():
        return g, False
    return torch.zeros_like(p, dtype=torch.float32 if p.dtype == torch.float32 else p.dtype), True


_DDP = []


def _notify(p):
    if not _DDP:
        from ..parallel import ddp

        _DDP.append(ddp.notify_grad_ready)
    _DDP[0](p)


class BertEmbeddings(nn.Module):
    def __init__(self, cfg, device=None):
        super().__init__()
        C = cfg.hidden_size
        std = cfg.initializer_range
        self.word = nn.Parameter(torch.randn(cfg.vocab_size, C, device=device) * std)
        self.pos = nn.Parameter(torch.randn(cfg.max_position_embeddings, C, device=device) * std)
        self.token_type = nn.Parameter(torch.randn(cfg.type_vocab_size, C, device=device) * std)
        self.ln_w = nn.Parameter(torch.ones(C, device=device))
        self.ln_b = nn.Parameter(torch.zeros(C, device=device))
        self.cfg = cfg


class BertLayer(nn.Module):
    def __init__(self, cfg, dtype=torch.bfloat16, device=None):
        super().__init__()
        C, I = cfg.hidden_size, cfg.intermediate_size
        std = cfg.initializer_range

        def w(o, i):
            return nn.Parameter((torch.randn(o, i, device=device) * std).to(dtype))

        def z(n):
            return nn.Parameter(torch.zeros(n, device=device))

        self.wqkv, self.bqkv = w(3 * C, C), z(3 * C)
        self.wo, self.bo = w(C, C), z(C)
        self.ln1_w, self.ln1_b = nn.Parameter(torch.ones(C, device=device)), z(C)
        self.w1, self.b1 = w(I, C), z(I)
        self.w2, self.b2 = w(C, I), z(C)
        self.ln2_w, self.ln2_b = nn.Parameter(torch.ones(C, device=device)), z(C)
        self.cfg = cfg

    def param_list(self):
        return [self.wqkv, self.bqkv, self.wo, self.bo, self.ln1_w, self.ln1_b, self.w1, self.b1, self.w2, self.b2,
                self.ln2_w, self.ln2_b]


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tts, emb, p, *params):
        cfg = emb.cfg
        B, S = ids.shape
        seed = next_seed() if p > 0 else 0
        h0 = raw.embed_sum(ids, tts, emb.word, emb.pos, emb.token_type, S)
        y, _, mean, rstd = raw.ln_fwd(h0, emb.ln_w, emb.ln_b, cfg.layer_norm_eps, p_out=p, seed_out=seed,
                                      keep_h=False)
        ctx.emb, ctx.p, ctx.seed, ctx.S = emb, p, seed, S
        ctx.save_for_backward(ids, tts, h0, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, tts, h0, mean, rstd = ctx.saved_tensors
        emb = ctx.emb
        owned = []
        sinks = {}
        for name in ("word", "pos", "token_type", "ln_w", "ln_b"):
            p = getattr(emb, name)
            g, own = _grad_out(p)
            sinks[name] = g
            owned.append(g if own else None)
        dh, _ = raw.ln_bwd(dy.contiguous(), h0, mean, rstd, emb.ln_w, sinks["ln_w"], sinks["ln_b"], p_out=ctx.p,
                           seed_out=ctx.seed)
        raw.embed_bwd(dh, ids, tts, sinks["word"], sinks["pos"], sinks["token_type"], ctx.S, emb.token_type.shape[0],
                      pad_id=emb.cfg.pad_token_id)
        for name in ("ln_b", "ln_w", "token_type", "pos", "word"):
            _notify(getattr(emb, name))
        # params order in apply(): word, pos, type, ln_w, ln_b
        return (None, None, None, None) + tuple(owned)


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, key_len, layer, B, S, p_hidden, p_attn, *params):
        cfg = layer.cfg
        H = cfg.num_attention_heads
        eps = cfg.layer_norm_eps
        sa = next_seed() if p_attn > 0 else 0
        s1 = next_seed() if p_hidden > 0 else 0
        s2 = next_seed() if p_hidden > 0 else 0
        qkv = raw.gemm(x, layer.wqkv, bias=layer.bqkv)
        ctx_, lse = raw.attn_fwd(qkv, B, S, H, key_len, p_attn, sa, scale=1.0 / math.sqrt(cfg.hidden_size // H))
        # the output projections' biases (bo, b2) are added by the LayerNorm pass that reads
        # their outputs (their gradients already come from its backward): the GEMMs are plain
        lnb = config.get("CLOUD_AMD_LN_BIAS_FWD")
        a = raw.gemm(ctx_, layer.wo, bias=None if lnb else layer.bo)
        y1, h1, m1, r1 = raw.ln_fwd(a, layer.ln1_w, layer.ln1_b, eps, residual=x, p_in=p_hidden, seed_in=s1,
                                    x_bias=layer.bo if lnb else None)
        del a
        pre = torch.empty((x.shape[0], cfg.intermediate_size), dtype=torch.bfloat16, device=x.device)
        f = raw.gemm(y1, layer.w1, bias=layer.b1, act=cfg.hidden_act, preact=pre)
        o = raw.gemm(f, layer.w2, bias=None if lnb else layer.b2)
        y2, h2, m2, r2 = raw.ln_fwd(o, layer.ln2_w, layer.ln2_b, eps, residual=y1, p_in=p_hidden, seed_in=s2,
                                    x_bias=layer.b2 if lnb else None)
        del o
        ctx.layer, ctx.B, ctx.S = layer, B, S
        ctx.cfgs = (p_hidden, p_attn, sa, s1, s2)
        ctx.save_for_backward(x, key_len, qkv, ctx_, lse, h1, m1, r1, y1, pre, f, h2, m2, r2)
        return y2

    @staticmethod
    def backward(ctx, dy2):
        layer = ctx.layer
        cfg = layer.cfg
        H = cfg.num_attention_heads
        B, S = ctx.B, ctx.S
        p_hidden, p_attn, sa, s1, s2 = ctx.cfgs
        x, key_len, qkv, ctx_, lse, h1, m1, r1, y1, pre, f, h2, m2, r2 = ctx.saved_tensors
        params = layer.param_list()
        sinks, owned = {}, []
        for p in params:
            g, own = _grad_out(p)
            sinks[id(p)] = g
            owned.append(g if own else None)

        def G(p):
            return sinks[id(p)]

        dy2 = dy2.contiguous()
        # weight / bias gradients (compute-bound GEMMs + column sums) go to the side
        # stream; the memory-bound LN / attention / dgrad chain stays on the main stream.
        # Their fixed-order finalisations (split-K slab sums, column-partial sums) are
        # batched into one launch at the end of the layer (raw.deferred_finalize), and
        # the DDP bucket notifications follow it.
        side = SideWork(dy2.device)
        main_ready, side_ready = [], []

        fuse_bias = config.get("CLOUD_AMD_LN_BIAS_SUM")

        def param_grads(dy, inp, w, b, bias_done=False):
            bias_done = bias_done and fuse_bias

            def fn():
                if not bias_done:
                    raw.colsum_into(dy, G(b))
                raw.wgrad_into(dy, inp, G(w))
            side.run(fn, dy, inp)
            (side_ready if side.enabled else main_ready).extend((w,) if bias_done else (b, w))

        with raw.deferred_finalize(enabled=config.get("CLOUD_AMD_GRAD_FIN_BATCH")):
            # LN2 (+ residual y1, + dropout on the FFN output); the same pass sums the
            # gradient it hands to the FFN output projection into b2's gradient
            dh2, do = raw.ln_bwd(dy2, h2, m2, r2, layer.ln2_w, G(layer.ln2_w), G(layer.ln2_b), p_in=p_hidden,
                                 seed_in=s2, want_dx=True, dsum=G(layer.b2) if fuse_bias else None)
            main_ready.extend((layer.ln2_b, layer.ln2_w))
            if fuse_bias:
                main_ready.append(layer.b2)
            param_grads(do, f, layer.w2, layer.b2, bias_done=True)
            dpre = raw.gemm(do, layer.w2, layout=raw.NN, act=cfg.hidden_act, dact_src=pre)
            del do, f
            param_grads(dpre, y1, layer.w1, layer.b1)
            raw.gemm(dpre, layer.w1, layout=raw.NN, out=dh2, beta=1.0)  # dy1 = dh2 + dpre W1
            del dpre
            dy1 = dh2
            # LN1 (+ residual x, + dropout on the attention output projection)
            dh1, da = raw.ln_bwd(dy1, h1, m1, r1, layer.ln1_w, G(layer.ln1_w), G(layer.ln1_b), p_in=p_hidden,
                                 seed_in=s1, want_dx=True, dsum=G(layer.bo) if fuse_bias else None)
            main_ready.extend((layer.ln1_b, layer.ln1_w))
            if fuse_bias:
                main_ready.append(layer.bo)
            del dy1
            param_grads(da, ctx_, layer.wo, layer.bo, bias_done=True)
            dctx = raw.gemm(da, layer.wo, layout=raw.NN)
            del da
            dqkv = raw.attn_bwd(qkv, ctx_, dctx, lse, B, S, H, key_len, p_attn, sa,
                                scale=1.0 / math.sqrt(cfg.hidden_size // H))
            del dctx
            param_grads(dqkv, x, layer.wqkv, layer.bqkv)
            raw.gemm(dqkv, layer.wqkv, layout=raw.NN, out=dh1, beta=1.0)  # dx = dh1 + dqkv Wqkv
        # (the batch flushed per stream on exit: LN finalisations on the main stream, the
        # weight-gradient / bias ones on the side stream behind their GEMMs)
        for p in main_ready:
            _notify(p)
        # the side stream's tail overlaps the next layer: its join + DDP notifications are
        # deferred one layer (side_stream.defer / settle; a backward callback settles all)
        side_stream.defer(side.detach(), side_ready, _notify)
        side_stream.settle(keep_last=1)
        return (dh1, None, None, None, None, None, None) + tuple(owned)


class _HeadFn(torch.autograd.Function):
    """logits = drop(tanh(h[:, 0] Wp^T + bp)) Wc^T + bc: the pooler GEMM reads the [CLS]
    rows in place (row stride S*C) with the tanh in its epilogue; dropout + the classifier
    (fp32 weights, fp32 logits) are one kernel forward and one backward (head.hip), the
    pooler's weight / bias gradient finalisations one batched launch."""

    @staticmethod
    def forward(ctx, h, wp, bp, wc, bc, B, S, p):
        C = h.shape[-1]
        cls = h.view(B, S * C)[:, :C]
        pooled = raw.gemm(cls, wp, bias=bp, act="tanh")
        seed = next_seed() if p > 0 else 0
        logits = raw.cls_head_fwd(pooled, wc, bc, p, seed)
        ctx.save_for_backward(h, pooled)
        ctx.B, ctx.S, ctx.p, ctx.seed = B, S, p, seed
        ctx.params = (wp, bp, wc, bc)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        h, pooled = ctx.saved_tensors
        B, S = ctx.B, ctx.S
        C = h.shape[-1]
        wp, bp, wc, bc = ctx.params
        sinks = [_grad_out(t) for t in (wp, bp, wc, bc)]
        (gw, _), (gb, _), (gwc, _), (gbc, _) = sinks
        dpre = raw.cls_head_bwd(dlogits, pooled, wc, gwc, gbc, ctx.p, ctx.seed)
        cls = h.view(B, S * C)[:, :C]
        with raw.deferred_finalize(enabled=config.get("CLOUD_AMD_GRAD_FIN_BATCH")):
            raw.wgrad_into(dpre, cls, gw)
            raw.colsum_into(dpre, gb)
        for t in (bc, wc, bp, wp):
            _notify(t)
        dh = torch.zeros_like(h)
        dcls = dh.view(B, S * C)[:, :C]
        raw.gemm(dpre, wp, layout=raw.NN, out=dcls)
        return (dh,) + tuple(g if own else None for g, own in sinks) + (None, None, None)


class BertForSequenceClassification(nn.Module):
    """BERT encoder + tanh pooler + linear classifier (``num_labels`` classes)."""

    def __init__(self, cfg: BertConfig = None, dtype=torch.bfloat16, device=None):
        super().__init__()
        cfg = cfg or BertConfig()
        assert cfg.hidden_size % cfg.num_attention_heads == 0
        self.cfg = cfg
        self.dtype = dtype
        self.embeddings = BertEmbeddings(cfg, device=device)
        self.layers = nn.ModuleList([BertLayer(cfg, dtype=dtype, device=device)
                                     for _ in range(cfg.num_hidden_layers)])
        C = cfg.hidden_size
        self.pool_w = nn.Parameter((torch.randn(C, C, device=device) * cfg.initializer_range).to(dtype))
        self.pool_b = nn.Parameter(torch.zeros(C, device=device))
        self.cls_w = nn.Parameter(torch.randn(cfg.num_labels, C, device=device) * cfg.initializer_range)
        self.cls_b = nn.Parameter(torch.zeros(cfg.num_labels, device=device))

    # ------------------------------------------------------------------ paths
    def _native_ok(self, input_ids):
        cfg = self.cfg
        return (input_ids.is_cuda and self.dtype == torch.bfloat16 and _ext.use_native(input_ids)
                and cfg.hidden_size // cfg.num_attention_heads == 64 and input_ids.shape[1] % 64 == 0
                and cfg.hidden_size % 8 == 0 and cfg.intermediate_size % 8 == 0)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None):
        """input_ids [B, S] -> logits [B, num_labels] (fp32)."""
        if self._native_ok(input_ids):
            return self._native_forward(input_ids, token_type_ids, attention_mask)
        return self._torch_forward(input_ids, token_type_ids, attention_mask)

    def _native_forward(self, input_ids, token_type_ids, attention_mask):
        cfg = self.cfg
        B, S = input_ids.shape
        train = self.training
        ph = cfg.hidden_dropout_prob if train else 0.0
        pa = cfg.attention_probs_dropout_prob if train else 0.0
        ids = input_ids.to(torch.int32).contiguous()
        tts = token_type_ids.to(torch.int32).contiguous() if token_type_ids is not None else torch.zeros_like(ids)
        key_len = (attention_mask.sum(1).to(torch.int32).contiguous() if attention_mask is not None else None)
        e = self.embeddings
        if torch.is_grad_enabled():
            side_stream.begin_pass()  # drop deferred state of a backward that raised
        h = _EmbedFn.apply(ids, tts, e, ph, e.word, e.pos, e.token_type, e.ln_w, e.ln_b)
        for layer in self.layers:
            h = _LayerFn.apply(h, key_len, layer, B, S, ph, pa, *layer.param_list())
        if self.cls_w.shape[0] <= _ext.load(required=True).cls_head_max_labels():
            return _HeadFn.apply(h, self.pool_w, self.pool_b, self.cls_w, self.cls_b, B, S, ph)
        pooled = torch.tanh(F.linear(h.view(B, S, -1)[:, 0].float(), self.pool_w.float(), self.pool_b))
        return F.linear(F.dropout(pooled, ph, train), self.cls_w, self.cls_b)

    def _torch_forward(self, input_ids, token_type_ids=None, attention_mask=None):
        """Plain PyTorch (fp32 math) -- CPU path and numerics reference."""
        cfg = self.cfg
        B, S = input_ids.shape
        C, H = cfg.hidden_size, cfg.num_attention_heads
        D = C // H
        train = self.training
        ph = cfg.hidden_dropout_prob if train else 0.0
        pa = cfg.attention_probs_dropout_prob if train else 0.0
        act = {"gelu": lambda t: F.gelu(t), "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"),
               "relu": F.relu}[cfg.hidden_act]
        e = self.embeddings
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
        pos = torch.arange(S, device=input_ids.device)
        x = F.embedding(input_ids, e.word, padding_idx=cfg.pad_token_id) + e.pos[pos][None] + e.token_type[tt]
        x = F.dropout(F.layer_norm(x, (C,), e.ln_w, e.ln_b, cfg.layer_norm_eps), ph, train)
        mask = None
        if attention_mask is not None:
            mask = (1.0 - attention_mask.float())[:, None, None, :] * -1e30
        for L in self.layers:
            qkv = F.linear(x, L.wqkv.float(), L.bqkv)
            q, k, v = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
            att = (q @ k.transpose(-1, -2)) / math.sqrt(D)
            if mask is not None:
                att = att + mask
            att = F.dropout(att.softmax(-1), pa, train)
            c = (att @ v).permute(0, 2, 1, 3).reshape(B, S, C)
            a = F.dropout(F.linear(c, L.wo.float(), L.bo), ph, train)
            x = F.layer_norm(x + a, (C,), L.ln1_w, L.ln1_b, cfg.layer_norm_eps)
            f = act(F.linear(x, L.w1.float(), L.b1))
            o = F.dropout(F.linear(f, L.w2.float(), L.b2), ph, train)
            x = F.layer_norm(x + o, (C,), L.ln2_w, L.ln2_b, cfg.layer_norm_eps)
        pooled = torch.tanh(F.linear(x[:, 0], self.pool_w.float(), self.pool_b))
        pooled = F.dropout(pooled, ph, train)
        return F.linear(pooled, self.cls_w, self.cls_b)


def bert_base(num_labels=2, **kw):
    return BertForSequenceClassification(BertConfig.base(num_labels=num_labels), **kw)
