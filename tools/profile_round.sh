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
#   pmc_sq/                 VALU / LDS-conflict / wait counters over PG iterations -> pmc_sq.json
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
if [ -z "${SKIP_PMC:-}" ]; then
  step pmc_fetch 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 tools/pmc_step.py
  step pmc_write 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 tools/pmc_step.py
  python tools/pmc_report.py "$O/pmc_fetch/**/*counter_collection.csv" "$O/pmc_write/**/*counter_collection.csv" 4194304 $O/pmc_step_kernel.json > /dev/null
  # this round's PMC file where bench.py reads roofline.traffic from (profiles/rNN/), so the bench
  # lines below cite traffic measured at the same HEAD
  mkdir -p profiles/${ROUND:-r05} && cp $O/pmc_step_kernel.json profiles/${ROUND:-r05}/pmc_step_kernel.json
  step pmc_mfma 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_mfma -o run -- python3 tools/prof_pg_iter.py
  python tools/pmc_kernels.py "$O/pmc_mfma/**/*counter_collection.csv" > $O/pmc_mfma.json
  # VALU / LDS / wait view of the same iterations (8 SQ counters: one pass)
  step pmc_sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 tools/prof_pg_iter.py
  python tools/pmc_kernels.py "$O/pmc_sq/**/*counter_collection.csv" > $O/pmc_sq.json
fi
CFGS=${CFGS-easy default hard_heldout variable_noise}  # CFGS="" skips the per-config lines
for c in $CFGS; do
  if [ "$c" = easy ]; then step bench_$c 300 python bench.py; else
    step bench_$c 200 python bench.py --config $c --no-cpu-baseline --no-roofline; fi
  grep '^{' $O/bench_$c.log > $O/bench_$c.json
  step prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
    python3 bench.py --config $c --no-cpu-baseline $( [ "$c" = easy ] || echo --no-roofline )
  grep '^{' $O/prof_$c.log > $O/prof_$c.json
done
# the extra lines: real PPO (4 epochs x 4 minibatches), C3 with progressions in every timed
# iteration, C3 under the reference's training-loop success rule, the RCCL path at world 1
if [ -z "${SKIP_EXTRA:-}" ]; then
  step bench_easy_ppo4x4 200 python bench.py --epochs 4 --minibatches 4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline
  grep '^{' $O/bench_easy_ppo4x4.log > $O/bench_easy_ppo4x4.json
  step prof_easy_ppo4x4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_easy_ppo4x4 -o run -- \
    python3 bench.py --epochs 4 --minibatches 4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline
  grep '^{' $O/prof_easy_ppo4x4.log > $O/prof_easy_ppo4x4.json
  # the cold-start C2 line: no clock prewarm before the warmup iterations
  step bench_easy_cold 200 python bench.py --prewarm-s 0 --no-cpu-baseline --no-roofline
  grep '^{' $O/bench_easy_cold.log > $O/bench_easy_cold.json
  step bench_default_restart 200 python bench.py --config default --sched-restart --no-cpu-baseline --no-roofline
  grep '^{' $O/bench_default_restart.log > $O/bench_default_restart.json
  step bench_default_training 200 python bench.py --config default --success-rule training --no-cpu-baseline --no-roofline
  grep '^{' $O/bench_default_training.log > $O/bench_default_training.json
  step bench_easy_dist 200 python bench.py --dist --no-cpu-baseline --no-roofline
  grep '^{' $O/bench_easy_dist.log > $O/bench_easy_dist.json
  step eval_bench 200 python tools/eval_bench.py
  grep '^{' $O/eval_bench.log > $O/eval_bench.jsonl
fi
# interleaved rollout A/B on one box (DESIGN §9 ratios): C2 easy (16-env kernel) and C5 variable +
# noise at 4096 envs, C4 hard at 8192 envs (32-env kernel; ws16 = the 16-env kernel forced)
if [ -z "${SKIP_RT:-}" ]; then
  for i in 1 2 3; do
    step rt_easy_$i 120 env CUR=easy DIAGS=0:ws python tools/rollout_time.py
    step rt_variable_$i 120 env CUR=variable DIAGS=0:ws python tools/rollout_time.py
    step rt_hard8192_$i 120 env CUR=hard ENVS=8192 DIAGS=0:e8,2048:ws16 python tools/rollout_time.py
  done
  grep -h -v amdgpu $O/rt_*.log > $O/rollout_ratio_ab.log
  step stamps_ws 120 python tools/rollout_stamps.py
  step stamps_e8 120 env ENVS=8192 python tools/rollout_stamps.py
fi
if [ -z "${SKIP_SWEEP:-}" ]; then step step_sweep 300 python tools/step_sweep.py 12 24; grep '^{' $O/step_sweep.log > $O/step_sweep.jsonl; fi
for c in $CFGS easy_ppo4x4; do
  f=$(ls $O/prof_$c/*kernel_trace.csv $O/prof_$c/*/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python tools/trace_summary.py "$f" > $O/trace_summary_$c.txt
done
echo done | tee -a $O/session.log
