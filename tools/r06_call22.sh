#!/bin/bash
# H2 DMA issue placement: parity of the in-layer-1 variants, stamps, iteration and kernel A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
for v in h2P1 h2P2; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "stored_h2" > gpurun_out/r06/pytest_$v.log 2>&1 || { tail -20 gpurun_out/r06/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r06/pytest_$v.log
done
for v in h2S h2S1 h2S2; do
  DXRL_LIB=ab/lib$v.so DXRL_FUSED_DIAG=8 VARIANT=both REPS=2 timeout -k 10 120 python tools/h2_stamps.py 2>&1 | grep "train=1" | sed "s/^/$v /" >> gpurun_out/r06/h2_stamps_place.log || exit 2
done
VARIANTS="h2P0 h2P1 h2P2" bash tools/ab.sh 3 tools/h2_ab.py || exit 3
VARIANTS="h2P0 h2P1 h2P2" bash tools/ab_kernels.sh 2 > gpurun_out/abk_summary.log 2>&1 || exit 4
cat gpurun_out/abk_summary.log
