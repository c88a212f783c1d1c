#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 ddp_backend.log env CLOUD_AMD_DDP_ORDER=backend python scripts/ddp_probe.py || exit 1
$S 300 ddp_event.log env CLOUD_AMD_DDP_ORDER=event python scripts/ddp_probe.py || exit 1
$S 300 ddp_event_big.log env CLOUD_AMD_DDP_ORDER=event PROBE_BUCKET_MB=1000 python scripts/ddp_probe.py || exit 1
$S 300 ddp_sync.log env CLOUD_AMD_DDP_ORDER=sync python scripts/ddp_probe.py || exit 1
$S 300 pytest_ddp_gpu.log python -m pytest tests/test_ddp_gpu.py -q || exit 1
echo SESSION_DONE
