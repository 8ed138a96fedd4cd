#!/bin/bash
# round-6 GPU call 9: k_wgrad_l1 with H1(c+1)'s tanh in chunk c's second k-step (DXRL_WL1_ILV):
# bit-exactness tests on the in-tree build, then the kernel-level A/B (N = interleaved, O = before)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_gemm.py tests/test_gpu_pg.py > gpurun_out/r06/pytest_wl1_ilv.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06/pytest_wl1_ilv.log; exit 3; }
tail -2 gpurun_out/r06/pytest_wl1_ilv.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="N O" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_wl1_ilv.log 2>&1 || exit 4
cat gpurun_out/r06/abk_wl1_ilv.log
