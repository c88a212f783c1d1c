"""Feasibility + timing probe: BERT-base training step eager vs captured in one HIP graph.

One process, one GPU, no run(): warm up eagerly, time K eager steps, capture the step
(forward, loss, backward, fused AdamW kernels with device hyper-parameters), time K replays.
Prints one JSON line.  Dropout seeds are whatever the capture froze (timing only).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.bert_base_synth import synthetic_glue  # noqa: E402
from cloud_amd.models.bert import BertConfig, BertForSequenceClassification  # noqa: E402
from cloud_amd.ops import softmax_cross_entropy  # noqa: E402
from cloud_amd.optim import AdamW  # noqa: E402


def main():
    steps = int(os.environ.get("STEPS", "30"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    B, S = 64, 128
    ids, tts, am, labels = synthetic_glue(B, S, dev, 1000)
    model = BertForSequenceClassification(BertConfig.base(num_labels=2), device=dev)
    opt = AdamW(model, learning_rate=2e-5, weight_decay=0.01)

    def fwd_bwd():
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(model(ids, tts, am), labels, denom=B)
        loss.backward()
        return loss

    def eager():
        loss = fwd_bwd()
        opt.step()
        return loss

    for _ in range(5):
        eager()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        th = time.perf_counter()
        eager()
        host.append((time.perf_counter() - th) * 1e3)
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t0) / steps * 1e3
    print("eager ok %.3f ms/step" % eager_ms, flush=True)

    opt.prepare_step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fwd_bwd()
            opt.step_kernels()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    print("capture...", flush=True)
    with torch.cuda.graph(g):
        loss_g = fwd_bwd()
        opt.step_kernels()
    torch.cuda.synchronize()
    print("captured", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ghost = []
    t0 = time.perf_counter()
    for _ in range(steps):
        th = time.perf_counter()
        g.replay()
        ghost.append((time.perf_counter() - th) * 1e3)
    torch.cuda.synchronize()
    graph_ms = (time.perf_counter() - t0) / steps * 1e3
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(json.dumps({"eager_ms": round(eager_ms, 3), "graph_ms": round(graph_ms, 3),
                      "eager_seq_s": round(B / eager_ms * 1e3, 1), "graph_seq_s": round(B / graph_ms * 1e3, 1),
                      "eager_host_median_ms": round(med(host), 3), "graph_host_median_ms": round(med(ghost), 3),
                      "loss_graph": float(loss_g.float())}), flush=True)


if __name__ == "__main__":
    main()
