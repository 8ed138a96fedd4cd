#!/bin/bash
# round-6 GPU call 2: changed tests again (kpartial setter), kernel-level A/B B vs G, stamps B vs G
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
: timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pg.py tests/test_gpu_fullsize.py \
  "tests/test_gpu_parity.py::test_streaming_step_policy_is_bit_identical" > gpurun_out/r06/pytest_call2.log 2>&1
rc=0
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="B G" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_early_w.log 2>&1 || exit 3
for v in B G; do for i in 1 2; do
  DXRL_LIB=ab/lib$v.so DXRL_FUSED_DIAG=8 REPS=2 timeout -k 10 120 python tools/prof_fused.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/stamps_early_w.log || exit 4
done; done
echo done
