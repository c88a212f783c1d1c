#!/usr/bin/env bash
# GPU tests after the round-2 test additions (optimizer parity vs torch.optim, DDP vs single process).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 r2s4_pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread || exit 1
echo SESSION_DONE
