#!/usr/bin/env bash
# Round-4 session 14: fused input+weight gradient kernels (stage-1 conv3 default; stage-1 conv1 and
# stage-2 conv3 opt-in) numerics; ResNet-50 A/B default / +conv1 / +stage-2 / GC freeze off (step
# probe in the JSON); serialized step profiles of default and of all fused paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s14}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold_tests.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold_tests.log
for i in 1 2; do
$S 240 ${tag}_def_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD1=1 $S 240 ${tag}_c1_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD2=1 $S 240 ${tag}_s2_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
CLOUD_AMD_GC_FREEZE=0 $S 240 ${tag}_nofreeze.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
for v in def all; do
rm -rf gpurun_out/${tag}_prof_$v
if [ $v = all ]; then export CLOUD_AMD_BN_FOLD_WGRAD1=1 CLOUD_AMD_BN_FOLD_WGRAD2=1; fi
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_$v.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_$v -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_$v sgd_kernel > gpurun_out/${tag}_rn_step_kernels_$v.txt
rm -rf gpurun_out/${tag}_prof_$v
head -3 gpurun_out/${tag}_rn_step_kernels_$v.txt
done
unset CLOUD_AMD_BN_FOLD_WGRAD1 CLOUD_AMD_BN_FOLD_WGRAD2
bash scripts/r3_prof_bert.sh ${tag} > gpurun_out/${tag}_bert_prof_session.log 2>&1 || { tail -20 gpurun_out/${tag}_bert_prof_session.log; exit 1; }
rm -rf gpurun_out/${tag}_prof_bert
for f in def_1 c1_1 s2_1 def_2 c1_2 s2_2 nofreeze; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
