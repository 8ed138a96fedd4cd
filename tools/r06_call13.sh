#!/bin/bash
# round-6 GPU call 13: the noise draws in the head phase (DXRL_WS_NOISE_IN_HEAD):
# tape / oracle tests on the in-tree build, then the rollout A/B (A = noise drawn in the head phase, P = in P0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_ablation.py tests/test_gpu_eval.py > gpurun_out/r06/pytest_noise_head.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_noise_head.log; exit 3; }
tail -2 gpurun_out/r06/pytest_noise_head.log
rm -f gpurun_out/ab.log
for i in 1 2 3 4; do
  for v in A P; do
    DXRL_LIB=ab/lib$v.so CUR=easy DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 4
    DXRL_LIB=ab/lib$v.so CUR=variable DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 4
  done
done
cp gpurun_out/ab.log gpurun_out/r06/ab_noise_head.log; cat gpurun_out/r06/ab_noise_head.log
