#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 ddp_probe.log python scripts/ddp_probe.py || exit 1
$S 300 ddp_probe_big.log env PROBE_BUCKET_MB=1000 python scripts/ddp_probe.py || exit 1
echo SESSION_DONE
