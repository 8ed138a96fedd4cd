#!/bin/bash
# GPU power and clocks sampled (rocm-smi, sysfs readers only) while bench.py runs a long C2 line and
# a long rollout-only loop, to see whether the iteration runs at the power limit
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rocm-smi --showmaxpower --showpower --showclocks > gpurun_out/r06/smi_idle.log 2>&1
( for i in $(seq 1 60); do echo "t=$i $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk|fclk|mclk" ; sleep 0.3; done ) > gpurun_out/r06/smi_bench.log 2>&1 &
mon=$!
timeout -k 10 200 python bench.py --steps 400 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r06/bench_long.log 2>&1; rc=$?
wait $mon
[ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/r06/bench_long.log | cut -c1-160
grep -c Power gpurun_out/r06/smi_bench.log
cat gpurun_out/r06/smi_idle.log | grep -E "Power|sclk|Max"
