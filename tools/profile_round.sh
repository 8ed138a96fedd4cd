#!/bin/bash
# One GPU session producing a round's evidence under gpurun_out/r/ (copy to profiles/rNN/):
#   bench_<cfg>.json        bench.py JSON line per BASELINE config (un-profiled)
#   prof_<cfg>/             rocprofv3 --kernel-trace --stats of bench.py (the same command);
#                           prof_<cfg>.json is the JSON line that profiled run printed, so the
#                           roofline line and the kernel stats come from one process
#   step_sweep.jsonl        k_step N = 2^12 .. 2^24
#   pmc_fetch/ pmc_write/   separate --pmc passes over k_step at 2^22 envs -> pmc_step_kernel.json
#   pmc_mfma/               SQ_INSTS_VALU_MFMA_MOPS_BF16 + SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
#                           over PG iterations -> pmc_mfma.json
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a $O/session.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -2 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc" | tee -a $O/session.log; exit $rc; fi
}
CFGS=${CFGS:-easy default hard_heldout variable_noise}
for c in $CFGS; do
  if [ "$c" = easy ]; then step bench_$c 300 python bench.py; else
    step bench_$c 200 python bench.py --config $c --no-cpu-baseline --no-roofline; fi
  grep '^{' $O/bench_$c.log > $O/bench_$c.json
  step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
    python3 bench.py --config $c --no-cpu-baseline $( [ "$c" = easy ] || echo --no-roofline )
  grep '^{' $O/prof_$c.log > $O/prof_$c.json
done
if [ -z "${SKIP_SWEEP:-}" ]; then step step_sweep 300 python tools/step_sweep.py 12 24; grep '^{' $O/step_sweep.log > $O/step_sweep.jsonl; fi
if [ -z "${SKIP_PMC:-}" ]; then
  step pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 tools/pmc_step.py
  step pmc_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 tools/pmc_step.py
  python tools/pmc_report.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" 4194304 $O/pmc_step_kernel.json > /dev/null
  step pmc_mfma 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_mfma -o run -- python3 tools/prof_pg_iter.py
  python tools/pmc_kernels.py "$O/pmc_mfma/**/*counter_collection.csv" > $O/pmc_mfma.json
fi
for c in $CFGS; do
  f=$(ls $O/prof_$c/*kernel_trace.csv $O/prof_$c/*/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python tools/trace_summary.py "$f" > $O/trace_summary_$c.txt
done
echo done | tee -a $O/session.log
