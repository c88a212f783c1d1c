"""hipBLASLt (torch.mm) comparator for bin/gemm_bench: the same shapes and layouts on
uniform [-1, 1) bf16 operands, one JSON line per shape.

    python bench/blas_ref.py 4096,4096,4096,0 8192,2304,768,0 ...   (layout 0 NT, 1 NN, 2 TN)
"""
import json
import sys

import torch


def main():
    torch.manual_seed(0)
    for arg in sys.argv[1:]:
        M, N, K, L = (int(v) for v in arg.split(","))
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        if L == 2:
            a = (torch.rand(K, M, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16) if L == 0 else \
            (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        if L == 0:
            fn = lambda: torch.mm(a, b.t())  # noqa: E731
        elif L == 1:
            fn = lambda: torch.mm(a, b)  # noqa: E731
        else:
            fn = lambda: torch.mm(a.t(), b)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        print(json.dumps({"variant": "hipblaslt", "M": M, "N": N, "K": K, "layout": L, "us": round(ms * 1e3, 1),
                          "TF": round(2.0 * M * N * K / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
