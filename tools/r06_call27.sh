#!/bin/bash
# the in-layer-1 H2 issue by waves 4..7 as the default build: GPU suite, smoke, kernel A/B against
# the tile-start DMA (h2P0) with rotated order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06/pytest_gpu_dma47.log 2>&1 || { tail -30 gpurun_out/r06/pytest_gpu_dma47.log; exit 1; }
tail -1 gpurun_out/r06/pytest_gpu_dma47.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke_dma47.log 2>&1 || exit 2
tail -1 gpurun_out/r06/smoke_dma47.log
i=0
for order in "h2P0 NEW" "NEW h2P0" "h2P0 NEW" "NEW h2P0"; do
  i=$((i+1))
  for v in $order; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/${v}_$i.log 2>&1 || exit 3
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"]/1e6,1), d["ms_per_step"])' >> gpurun_out/r06/dma47_bench.log
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/abk_summary.log
cat gpurun_out/r06/dma47_bench.log gpurun_out/abk_summary.log
