"""Which ResNet gradient slots differ between the transform-A tile modes (CLOUD_AMD_XA_N256
0 / 1 / 2) with every BN fold site on?  Diagnostic for the 128 x 256 tiles."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["CLOUD_AMD_BN_FOLD_ALL"] = "1"
import torch  # noqa: E402

from cloud_amd.models.resnet import ResNet  # noqa: E402
from cloud_amd.ops import _ext, softmax_cross_entropy  # noqa: E402
from cloud_amd.optim import SGD  # noqa: E402

ext = _ext.load(required=True)


def grads(mode):
    ext.gemm_set_xa_n256(mode)
    torch.manual_seed(0)
    m = ResNet((2, 2, 2, 1), num_classes=10, stem_channels_pad=5, device="cuda")
    opt = SGD(m, learning_rate=0.05, momentum=0.9)
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(16, 64, 64, 3, device="cuda", generator=g).to(torch.bfloat16)
    Y = torch.randint(0, 10, (16,), device="cuda", generator=g)
    opt.zero_grad()
    loss, _ = softmax_cross_entropy(m(X), Y, denom=16)
    loss.backward()
    torch.cuda.synchronize()
    return [a.grad.detach().clone() for a in opt.arenas], [[(s.name, s.offset, s.numel) for s in a.slots] for a in opt.arenas]


g0, names = grads(0)
for mode in (1, 2):
    g1, _ = grads(mode)
    for ai, (x, y) in enumerate(zip(g1, g0)):
        bad = [(n, k, float((x[o:o + k].float() - y[o:o + k].float()).abs().max())) for n, o, k in names[ai]
               if not torch.equal(x[o:o + k], y[o:o + k])]
        print("mode", mode, "arena", ai, x.dtype, "differing slots (backward order last):", bad if ai else bad[-6:], len(bad))
