#!/bin/bash
# k_pg_values: the critic's H2 rows stored by waves 4..7 only (VH) vs every wave (NEW): parity and
# kernel A/B with rotated order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
DXRL_LIB=ab/libVH.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "stored_h2 or values" > gpurun_out/r06/pytest_VH.log 2>&1 || { tail -20 gpurun_out/r06/pytest_VH.log; exit 1; }
tail -1 gpurun_out/r06/pytest_VH.log
i=0
for order in "NEW VH" "VH NEW" "NEW VH" "VH NEW"; do
  i=$((i+1))
  for v in $order; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/${v}_$i.log 2>&1 || exit 3
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"]/1e6,1), d["ms_per_step"])' >> gpurun_out/r06/vh_bench.log
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/abk_summary.log
cat gpurun_out/r06/vh_bench.log gpurun_out/abk_summary.log
