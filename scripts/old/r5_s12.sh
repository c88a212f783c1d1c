#!/usr/bin/env bash
# Round-5 session 12: full GPU suite + smoke on the tree with the halo convolutions, the
# one-launch BN finalize and the 256 x 96 GEMM tiles; ResNet-50 and BERT benches; BERT profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s12}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 1100 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
chk ${tag}_all.log
tail -3 gpurun_out/${tag}_all.log
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
tail -2 gpurun_out/${tag}_smoke.log
$S 300 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 ${tag}_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
rm -rf gpurun_out/${tag}_bprof
$S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
for f in gpurun_out/${tag}_rn.log gpurun_out/${tag}_bert.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
head -14 gpurun_out/${tag}_bert_step_kernels.txt
echo SESSION_DONE
