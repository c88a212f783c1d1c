"""Test workload: each rank all-reduces its rank id and writes what it saw."""
import json
import os
import sys

import torch

import cloud_amd.parallel.strategy as S

strategy = S.get_strategy()
r = strategy.reduce(S.ReduceOp.SUM, torch.tensor([float(strategy.rank + 1)]))
out = {
    "rank": strategy.rank, "replicas": strategy.num_replicas_in_sync, "sum": float(r[0]),
    "strategy": type(strategy).__name__, "tf_config": json.loads(os.environ.get("TF_CONFIG", "{}")),
    "remote": os.environ.get("TF_KERAS_RUNNING_REMOTELY"), "argv": sys.argv[1:],
    "device": str(strategy.device),
}
print("RESULT " + json.dumps(out), flush=True)
if os.environ.get("FAIL_RANK") == str(strategy.rank):
    sys.exit(3)
