#!/bin/bash
# One GPU session producing the round's evidence under gpurun_out/:
#   bench.log        bench.py JSON line (default workload)
#   prof/            rocprofv3 --kernel-trace --stats of bench.py (same command, fewer steps)
#   pmc_fetch/, pmc_write/  separate --pmc passes over k_step at 2^22 envs
#   pmc_step_kernel.json    corrected HBM bytes per launch (tools/pmc_report.py)
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $O/profile_round.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc" | tee -a $O/profile_round.log; exit $rc; fi
}
step bench 400 python bench.py ${BENCH_ARGS:-}
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
step pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 tools/pmc_step.py
step pmc_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 tools/pmc_step.py
python tools/pmc_report.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" 4194304 $O/pmc_step_kernel.json > /dev/null
python tools/trace_summary.py $(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/trace_summary.txt
echo done
