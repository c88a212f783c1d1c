"""Diagnostic (not a test): per-parameter differences between whole-arena and per-bucket
AdamW steps on BERT-2L at world 1, after one and after several steps."""
import gc
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def run(sliced, steps):
    from cloud_amd.models.bert import BertConfig, BertForSequenceClassification
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import AdamW
    from cloud_amd.parallel.ddp import GradAllReducer

    torch.manual_seed(0)
    cfg = BertConfig.base(num_hidden_layers=2, num_labels=2, hidden_dropout_prob=0.0,
                          attention_probs_dropout_prob=0.0)  # (dropout seeds advance a global counter)
    m = BertForSequenceClassification(cfg, device="cuda")
    opt = AdamW(m, learning_rate=1e-3, weight_decay=0.01)
    red = GradAllReducer(opt.arenas, world=1, bucket_mb=4.0)
    if sliced:
        assert red.attach_optimizer(opt)
    g = torch.Generator(device="cuda").manual_seed(7)
    # unique token ids: the word-embedding gradient rows then take one (atomic) contribution each
    ids = (torch.randperm(29000, device="cuda", generator=g)[:16 * 128] + 1000).view(16, 128)
    tts = torch.zeros_like(ids)
    am = torch.ones_like(ids)
    labels = torch.randint(0, 2, (16,), device="cuda", generator=g)
    grads = None
    for i in range(steps):
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m(ids, tts, am), labels, denom=16)
        loss.backward()
        red.finish()
        if i == steps - 1:
            torch.cuda.synchronize()
            grads = [a.grad.detach().clone() for a in opt.arenas]
        opt.step()
    torch.cuda.synchronize()
    names = [n for n, _ in m.named_parameters()]
    out = ([p.detach().clone() for p in m.parameters()], grads, float(loss.detach()), names,
           [len(b.slots) for b in red.buckets], red.buckets and [(b.arena is opt.arenas[0], b.lo, b.hi) for b in red.buckets])
    del m, opt, red
    gc.collect()
    return out


for steps in (1, 2):
    A = run(False, steps)
    A2 = run(False, steps)
    S = run(True, steps)
    print("steps", steps, "loss base/base2/sliced", A[2], A2[2], S[2])
    print("buckets", S[4], S[5])
    for ai, (ga, gs) in enumerate(zip(A[1], S[1])):
        d = (ga.float() - gs.float()).abs()
        print("arena", ai, "grad maxdiff", float(d.max()), "nonzero diffs", int((d > 0).sum()), "of", d.numel())
    for n, a, a2, s in zip(A[3], A[0], A2[0], S[0]):
        d0 = float((a.float() - a2.float()).abs().max())
        d1 = float((a.float() - s.float()).abs().max())
        if d0 or d1:
            print("  %-40s base-vs-base %.3e  base-vs-sliced %.3e" % (n, d0, d1))
