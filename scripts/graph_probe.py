"""Find where HIP-graph capture of the training step breaks: capture progressively
larger pieces in ONE process, printing a line before/after each stage (the last
line before a crash names the culprit)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.models.resnet import ResNet  # noqa: E402
from cloud_amd.ops import raw, softmax_cross_entropy  # noqa: E402
from cloud_amd.optim import SGD  # noqa: E402


def cap(name, fn):
    print("stage", name, "capture...", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    print("stage", name, "ok", flush=True)
    return g, out


def main():
    dev = "cuda"
    a = torch.randn(512, 256, device=dev).to(torch.bfloat16)
    w = torch.randn(128, 256, device=dev).to(torch.bfloat16)
    cap("gemm", lambda: raw.gemm(a, w))
    x = torch.randn(4, 16, 16, 64, device=dev).to(torch.bfloat16)
    wc = torch.randn(64, 3, 3, 64, device=dev).to(torch.bfloat16)
    cap("conv", lambda: raw.conv_fwd(x, wc, 1, 1))
    torch.manual_seed(0)
    m = ResNet((1, 1, 1, 1), num_classes=10, stem_channels_pad=5, device=dev)
    opt = SGD(m, learning_rate=0.01, momentum=0.9)
    xi = torch.randn(8, 32, 32, 3, device=dev).to(torch.bfloat16)
    yi = torch.randint(0, 10, (8,), device=dev)
    with torch.no_grad():
        cap("fwd_nograd", lambda: m(xi))

    def fwd_bwd():
        loss, _ = softmax_cross_entropy(m(xi), yi, denom=8)
        loss.backward()
        return loss.detach()

    def step():
        opt.zero_grad()
        out = fwd_bwd()
        opt.step_kernels()
        return out

    opt.prepare_step()
    cap("fwd_bwd", lambda: (opt.zero_grad(), fwd_bwd())[1])
    cap("step", step)
    print("ALL_STAGES_OK", flush=True)


if __name__ == "__main__":
    main()
