#!/bin/bash
# round-6 GPU call 3: learner variants kernel-level A/B + LDS-conflict PMC (B vs H)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="B H I K S T" bash tools/ab_kernels.sh 2 > gpurun_out/r06/abk_learner_variants.log 2>&1 || exit 3
for v in B S; do
  DXRL_LIB=ab/lib$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r06/pmc_sq_$v -o run -- python3 tools/prof_pg_iter.py > gpurun_out/r06/pmc_sq_$v.log 2>&1 || exit 4
  python tools/pmc_kernels.py "gpurun_out/r06/pmc_sq_$v/**/*counter_collection.csv" > gpurun_out/r06/pmc_sq_$v.json
done
echo done
