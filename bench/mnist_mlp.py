#!/usr/bin/env python3
"""BASELINE.json config 1: the README MNIST MLP launched through run() on a CPU
chief (OneDevice-equivalent) -- plumbing benchmark: end-to-end success,
run()->job-done wall time and training samples/s reported by the job.

    python bench/mnist_mlp.py [--epochs 2]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=2)
    args = ap.parse_args()
    import cloud_amd as tfc

    jobs = tempfile.mkdtemp(prefix="mlp_bench_")
    os.environ["MLP_EPOCHS"] = str(args.epochs)
    os.environ.setdefault("CLOUD_AMD_DEVICE", "cpu")
    os.chdir(os.path.join(ROOT, "examples", "workloads"))
    t0 = time.time()
    job = tfc.run(entry_point="mnist_example_using_fit_no_reqs.py", chief_config=tfc.COMMON_MACHINE_CONFIGS["CPU"],
                  jobs_dir=jobs, exit=False, wait=True, stream_logs=False)
    rc = job.wait()
    wall = time.time() - t0
    res = {}
    for log in glob.glob(os.path.join(job.job_dir, "logs", "*.log")):
        for ln in open(log):
            if ln.startswith("RESULT mlp"):
                res = dict(kv.split("=") for kv in ln.split()[2:])
    print(json.dumps({
        "metric": "samples/sec MNIST 2-layer MLP via run() on CPU (OneDevice)",
        "value": float(res.get("samples_per_s", 0.0)), "unit": "samples/sec", "n_gpus": 0,
        "success": rc == 0 and bool(res), "run_to_done_s": round(wall, 3), "fit_s": float(res.get("fit_s", 0.0)),
        "final_loss": float(res.get("loss", "nan")), "higher_is_better": True, "data": "synthetic MNIST (60000)",
        "config": {"model": "mlp-512-dropout0.2-10", "epochs": args.epochs, "batch": 128, "optimizer": "adam"},
        "job_id": job.job_id}), flush=True)
    sys.exit(0 if rc == 0 else 1)


if __name__ == "__main__":
    main()
