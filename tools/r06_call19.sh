#!/bin/bash
# round-6 GPU call 19: the rollout's H2 tape stored non-temporal (R, in-tree) vs plain (N, HEAD);
# iteration A/B (tools/h2_ab.py, both) interleaved x4, then the kernel view
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/ab_h2_tape_nt.log
for i in 1 2 3 4; do
  for v in R N; do
    DXRL_LIB=ab/lib$v.so VARIANT=both timeout -k 10 120 python tools/h2_ab.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/ab_h2_tape_nt.log || exit 4
  done
done
cat gpurun_out/r06/ab_h2_tape_nt.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="R N" bash tools/ab_kernels.sh 2 > gpurun_out/r06/abk_h2_tape_nt.log 2>&1 || exit 5
cat gpurun_out/r06/abk_h2_tape_nt.log
