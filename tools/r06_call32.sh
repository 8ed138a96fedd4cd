#!/bin/bash
# 16-byte epilogue stores (EB, -DDXRL_EPI_B128=1) vs the 8-byte ones (NEW): the whole GPU suite on
# EB, then kernel A/B with rotated order and the PMC LDS view of EB
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
DXRL_LIB=ab/libEB.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06/pytest_EB.log 2>&1 || { tail -30 gpurun_out/r06/pytest_EB.log; exit 1; }
tail -1 gpurun_out/r06/pytest_EB.log
i=0
for order in "NEW EB" "EB NEW" "NEW EB" "EB NEW"; do
  i=$((i+1))
  for v in $order; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/${v}_$i.log 2>&1 || exit 3
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"]/1e6,1), d["ms_per_step"])' >> gpurun_out/r06/eb_bench.log
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/abk_summary.log
for v in NEW EB; do
  DXRL_LIB=ab/lib$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_$v -o run -- python3 tools/prof_pg_iter.py > gpurun_out/r06/pmc_$v.log 2>&1 || exit 4
  python3 tools/pmc_kernels.py "gpurun_out/pmc_$v/**/*counter_collection.csv" > gpurun_out/r06/pmc_sq_$v.json
  python3 tools/pmc_table.py gpurun_out/r06/pmc_sq_$v.json fused values | sed "s/^/$v /" >> gpurun_out/r06/eb_pmc.log
done
cat gpurun_out/r06/eb_bench.log gpurun_out/abk_summary.log gpurun_out/r06/eb_pmc.log
