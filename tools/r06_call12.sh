#!/bin/bash
# round-6 GPU call 12: the noisy observation row written by the aux lanes (DXRL_WS_OBS_AUX):
# tape / oracle tests on the in-tree build, then the rollout A/B (A = aux-written row, P = before)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_ablation.py tests/test_gpu_eval.py > gpurun_out/r06/pytest_obs_aux.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_obs_aux.log; exit 3; }
tail -2 gpurun_out/r06/pytest_obs_aux.log
rm -f gpurun_out/ab.log
for i in 1 2 3 4; do
  for v in A P; do
    DXRL_LIB=ab/lib$v.so CUR=easy DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 4
    DXRL_LIB=ab/lib$v.so CUR=variable DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 4
  done
done
cp gpurun_out/ab.log gpurun_out/r06/ab_obs_aux.log; cat gpurun_out/r06/ab_obs_aux.log
