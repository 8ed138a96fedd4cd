#!/bin/bash
# H2 rows through registers (mode 4): parity, stamps, iteration and kernel A/B against the tile-start DMA
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
rm -f gpurun_out/ab.log
DXRL_LIB=ab/libh2P4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "stored_h2" > gpurun_out/r06/pytest_h2P4.log 2>&1 || { tail -20 gpurun_out/r06/pytest_h2P4.log; exit 1; }
tail -1 gpurun_out/r06/pytest_h2P4.log
for v in h2S h2S4; do
  DXRL_LIB=ab/lib$v.so DXRL_FUSED_DIAG=8 VARIANT=both REPS=2 timeout -k 10 120 python tools/h2_stamps.py 2>&1 | grep "train=1" | sed "s/^/$v /" >> gpurun_out/r06/h2_stamps_m4.log || exit 2
done
VARIANTS="h2P0 h2P4" bash tools/ab.sh 4 tools/h2_ab.py || exit 3
VARIANTS="h2P0 h2P4" bash tools/ab_kernels.sh 3 > gpurun_out/abk_summary.log 2>&1 || exit 4
cat gpurun_out/abk_summary.log
