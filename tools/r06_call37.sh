#!/bin/bash
# 32-env kernel's layer-2 tape copied by the aux waves in P4 (E8B) vs by every wave in the head
# phase (E8A): parity on E8B, e8 stamps, C4 rollout and iteration times interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
DXRL_LIB=ab/libE8B.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py > gpurun_out/r06/pytest_E8B.log 2>&1 || { tail -30 gpurun_out/r06/pytest_E8B.log; exit 1; }
tail -1 gpurun_out/r06/pytest_E8B.log
for v in E8A E8B; do
  DXRL_LIB=ab/lib$v.so ENVS=8192 timeout -k 10 120 python tools/rollout_stamps.py 2>&1 | grep -v amdgpu | head -12 | sed "s/^/$v /" >> gpurun_out/r06/e8b_stamps.log || exit 2
done
for i in 1 2 3; do for v in E8A E8B; do
  DXRL_LIB=ab/lib$v.so CUR=hard ENVS=8192 DIAGS=0:e8 timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/e8b_rt.log || exit 3
  DXRL_LIB=ab/lib$v.so VARIANT=tape timeout -k 10 150 python tools/e8_tape_ab.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/e8b_iter.log || exit 4
done; done
cat gpurun_out/r06/e8b_stamps.log gpurun_out/r06/e8b_rt.log gpurun_out/r06/e8b_iter.log
