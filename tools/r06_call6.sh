#!/bin/bash
# round-6 GPU call 6: L1 5:3 split A/B (kernel level) + stamps of both
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="I X" bash tools/ab_kernels.sh 4 > gpurun_out/r06/abk_l1split.log 2>&1 || exit 3
for v in I X; do
  DXRL_LIB=ab/lib$v.so DXRL_FUSED_DIAG=8 REPS=2 timeout -k 10 120 python tools/prof_fused.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/stamps_l1split.log || exit 4
done
echo done
