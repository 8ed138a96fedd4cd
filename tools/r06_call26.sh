#!/bin/bash
# mode 4 at 17 pieces per step with the pre-head vmcnt(0) on the issuing waves only (h2P4w) vs on
# every wave (h2P4p17) vs the tile-start DMA (h2P0): parity, stamps, kernel A/B with rotated order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
DXRL_LIB=ab/libh2P4w.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "stored_h2" > gpurun_out/r06/pytest_h2P4w.log 2>&1 || { tail -20 gpurun_out/r06/pytest_h2P4w.log; exit 1; }
tail -1 gpurun_out/r06/pytest_h2P4w.log
for v in h2S4p17 h2S4w; do
  DXRL_LIB=ab/lib$v.so DXRL_FUSED_DIAG=8 VARIANT=both REPS=2 timeout -k 10 120 python tools/h2_stamps.py 2>&1 | grep "train=1" | sed "s/^/$v /" >> gpurun_out/r06/h2_stamps_m4w.log || exit 2
done
i=0
for order in "h2P0 h2P4p17 h2P4w" "h2P4w h2P4p17 h2P0" "h2P4p17 h2P0 h2P4w" "h2P4w h2P0 h2P4p17"; do
  i=$((i+1))
  for v in $order; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/${v}_$i.log 2>&1 || exit 3
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"]/1e6,1), d["ms_per_step"])' >> gpurun_out/r06/m4w_bench.log
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/abk_summary.log
cat gpurun_out/r06/m4w_bench.log gpurun_out/abk_summary.log
