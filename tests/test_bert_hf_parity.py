"""BERT parity against an independent implementation: HuggingFace ``transformers``
``BertForSequenceClassification`` (importable offline here) loaded with the same random
weights.  On the CPU the PyTorch path of ``cloud_amd.models.bert`` must match HF in
fp32; on the GPU the native bf16 path (fused layer kernels, flash-style attention,
MFMA GEMM epilogues) must match HF-in-fp32 logits, loss and every parameter gradient
to bf16 tolerance.  Dropout off (eval-mode numerics) so both sides are deterministic."""
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")

from cloud_amd.models.bert import BertConfig, BertForSequenceClassification  # noqa: E402


def _pair(device, dtype, layers=2, hidden=128, heads=2, inter=512, vocab=512):
    cfg = BertConfig(vocab_size=vocab, hidden_size=hidden, num_hidden_layers=layers, num_attention_heads=heads,
                     intermediate_size=inter, max_position_embeddings=128, num_labels=3,
                     hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    ours = BertForSequenceClassification(cfg, dtype=dtype, device=device)
    hf_cfg = transformers.BertConfig(vocab_size=vocab, hidden_size=hidden, num_hidden_layers=layers,
                                     num_attention_heads=heads, intermediate_size=inter, max_position_embeddings=128,
                                     num_labels=3, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                                     layer_norm_eps=cfg.layer_norm_eps, hidden_act="gelu")
    hf = transformers.BertForSequenceClassification(hf_cfg).to(device).float()
    pairs = _mapping(ours, hf)
    with torch.no_grad():
        for get_ours, hf_param in pairs:
            hf_param.copy_(get_ours().float())
    return ours, hf, pairs


def _mapping(ours, hf):
    """(callable returning our tensor in HF's layout, HF parameter)."""
    C = ours.cfg.hidden_size
    e, he = ours.embeddings, hf.bert.embeddings
    m = [(lambda: e.word, he.word_embeddings.weight), (lambda: e.pos, he.position_embeddings.weight),
         (lambda: e.token_type, he.token_type_embeddings.weight), (lambda: e.ln_w, he.LayerNorm.weight),
         (lambda: e.ln_b, he.LayerNorm.bias)]
    for L, H in zip(ours.layers, hf.bert.encoder.layer):
        att = H.attention.self
        for i, lin in enumerate((att.query, att.key, att.value)):
            m.append((lambda L=L, i=i: L.wqkv[i * C:(i + 1) * C], lin.weight))
            m.append((lambda L=L, i=i: L.bqkv[i * C:(i + 1) * C], lin.bias))
        m += [(lambda L=L: L.wo, H.attention.output.dense.weight), (lambda L=L: L.bo, H.attention.output.dense.bias),
              (lambda L=L: L.ln1_w, H.attention.output.LayerNorm.weight),
              (lambda L=L: L.ln1_b, H.attention.output.LayerNorm.bias),
              (lambda L=L: L.w1, H.intermediate.dense.weight), (lambda L=L: L.b1, H.intermediate.dense.bias),
              (lambda L=L: L.w2, H.output.dense.weight), (lambda L=L: L.b2, H.output.dense.bias),
              (lambda L=L: L.ln2_w, H.output.LayerNorm.weight), (lambda L=L: L.ln2_b, H.output.LayerNorm.bias)]
    m += [(lambda: ours.pool_w, hf.bert.pooler.dense.weight), (lambda: ours.pool_b, hf.bert.pooler.dense.bias),
          (lambda: ours.cls_w, hf.classifier.weight), (lambda: ours.cls_b, hf.classifier.bias)]
    return m


def _our_grad(ours, get):
    """Gradient of our tensor `get()` -- slices of wqkv/bqkv map to slices of their grads."""
    t = get()
    base = t if t._base is None else t._base
    g = base.grad
    if t._base is None:
        return g
    off = t.storage_offset() - base.storage_offset()
    return g.reshape(-1)[off:off + t.numel()].view_as(t)


def _inputs(device, B=4, S=64, vocab=512):
    g = torch.Generator(device="cpu").manual_seed(3)
    ids = torch.randint(1, vocab, (B, S), generator=g)
    lens = torch.tensor([S, S - 5, S // 2 + 3, S // 2])[:B]
    am = (torch.arange(S)[None] < lens[:, None]).long()
    ids = ids * am
    tts = ((torch.arange(S)[None] >= (lens // 2)[:, None]) & (am == 1)).long()
    labels = torch.randint(0, 3, (B,), generator=g)
    return ids.to(device), tts.to(device), am.to(device), labels.to(device)


def _hf_step(hf, ids, tts, am, labels):
    hf.eval()
    hf.zero_grad()
    logits = hf(input_ids=ids, token_type_ids=tts, attention_mask=am).logits
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    return logits.detach(), loss.detach()


def test_torch_path_matches_hf_fp32_cpu():
    ours, hf, pairs = _pair("cpu", torch.float32)
    ids, tts, am, labels = _inputs("cpu")
    ref_logits, ref_loss = _hf_step(hf, ids, tts, am, labels)
    ours.eval()
    logits = ours(ids, tts, am)
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    torch.testing.assert_close(logits, ref_logits, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(loss, ref_loss, atol=1e-5, rtol=1e-5)
    for get, hp in pairs:
        torch.testing.assert_close(_our_grad(ours, get).float(), hp.grad, atol=1e-5, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dims", ["tiny", "base"])
def test_native_bf16_path_matches_hf_fp32_gpu(dims):
    """tiny: 2 x 128, 2 heads, seq 64; base: BERT-base, 12 layers x 768, 12 heads,
    3072 FFN, 30522 vocab, seq 128 (the benchmarked configuration)."""
    from cloud_amd.ops import _ext

    _ext.load(required=True)
    if dims == "base":
        ours, hf, pairs = _pair("cuda", torch.bfloat16, layers=12, hidden=768, heads=12, inter=3072, vocab=30522)
        ids, tts, am, labels = _inputs("cuda", S=128, vocab=30522)
    else:
        ours, hf, pairs = _pair("cuda", torch.bfloat16)
        ids, tts, am, labels = _inputs("cuda")
    assert ours._native_ok(ids)
    ref_logits, ref_loss = _hf_step(hf, ids, tts, am, labels)
    ours.eval()
    logits = ours(ids, tts, am)
    loss = F.cross_entropy(logits.float(), labels)
    loss.backward()
    torch.testing.assert_close(logits.float(), ref_logits, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(loss, ref_loss, atol=2e-2, rtol=2e-2)
    key_bias = {id(H.attention.self.key.bias) for H in hf.bert.encoder.layer}
    q_scale = max(float(H.attention.self.query.bias.grad.norm()) for H in hf.bert.encoder.layer)
    worst, bad = [], []
    for idx, (get, hp) in enumerate(pairs):
        g = _our_grad(ours, get).float()
        if id(hp) in key_bias:
            # the key-projection bias has an exactly-zero true gradient (softmax is invariant
            # to a per-query constant): HF's is fp32 round-off, ours bf16 round-off -- both must
            # be negligible next to the query-bias gradient, which flows through the same scores
            rel = float(g.norm()) / max(q_scale, 1e-12)
        else:
            rel = float((g - hp.grad).norm() / hp.grad.norm().clamp_min(1e-6))
        worst.append(rel)
        if rel >= 3e-2:
            bad.append((idx, tuple(hp.shape), rel))
    print("worst relative gradient error (%s): %.3e" % (dims, max(worst)))
    assert not bad, (dims, bad)
