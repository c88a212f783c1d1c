"""Per-parameter gradient error of the native BERT path vs HF and vs its own torch path."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch, torch.nn.functional as F
import test_bert_hf_parity as T

ours, hf, pairs = T._pair("cuda", torch.bfloat16)
ids, tts, am, labels = T._inputs("cuda")
ref_logits, ref_loss = T._hf_step(hf, ids, tts, am, labels)
ours.eval()
logits = ours(ids, tts, am)
F.cross_entropy(logits.float(), labels).backward()
nat = [T._our_grad(ours, g).float().clone() for g, _ in pairs]
for p in ours.parameters():
    p.grad = None
lt = ours._torch_forward(ids, tts, am)
F.cross_entropy(lt.float(), labels).backward()
tor = [T._our_grad(ours, g).float().clone() for g, _ in pairs]
print("logits", (logits.float() - ref_logits).abs().max().item(), (lt.float() - ref_logits).abs().max().item())
for i, ((g, hp), a, b) in enumerate(zip(pairs, nat, tor)):
    h = hp.grad
    r1 = float((a - h).norm() / h.norm().clamp_min(1e-12))
    r2 = float((b - h).norm() / h.norm().clamp_min(1e-12))
    r3 = float((a - b).norm() / b.norm().clamp_min(1e-12))
    print(i, tuple(h.shape), "nat-hf %.3g torch-hf %.3g nat-torch %.3g |h| %.3g |nat| %.3g" % (r1, r2, r3, h.norm(), a.norm()))
