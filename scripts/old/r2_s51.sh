#!/usr/bin/env bash
# Batch sweeps on the final kernels: ResNet-50 b512 / b2048 (buffer-window guards at 82 GB), BERT b128 / b256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 r2s51_resnet_b512.log python bench.py --via-run 0 --batch 512 || exit 1
$S 400 r2s51_resnet_b2048.log python bench.py --via-run 0 --batch 2048 --steps 10 --warmup 3 || exit 1
$S 300 r2s51_bert_b128.log python bench/bert_base_synth.py --via-run 0 --batch 128 || exit 1
$S 300 r2s51_bert_b256.log python bench/bert_base_synth.py --via-run 0 --batch 256 || exit 1
echo SESSION_DONE
