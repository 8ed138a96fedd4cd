#!/bin/bash
# round-6 GPU call 8: the two-tile pipelined learner (k_pg_dual) -- parity against k_pg_fused,
# then a kernel-level A/B (DXRL_FUSED_DUAL=1 vs 0, same library), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "two_tile" > gpurun_out/r06/pytest_dual.log 2>&1 || { echo "dual test failed"; tail -30 gpurun_out/r06/pytest_dual.log; exit 3; }
tail -3 gpurun_out/r06/pytest_dual.log
for i in 1 2 3; do
  for v in 1 0; do
    DXRL_FUSED_DUAL=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/dual${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/dual${v}_$i.log 2>&1 || exit 4
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/r06/abk_dual.log 2>&1
cat gpurun_out/r06/abk_dual.log
