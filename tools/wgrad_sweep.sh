#!/bin/bash
# k_wgrad_l1 per variant library (ab/lib<V>.so) and DXRL_WGRAD_DIAG ablation (0 full, 3 stream
# only): rocprofv3 kernel stats over short bench runs; prints the average k_wgrad_l1 duration.
#   VARIANTS="W3 W4" DIAGS="0 3" bash tools/wgrad_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ws
for v in ${VARIANTS:-W4}; do
  for d in ${DIAGS:-0 3}; do
    o=gpurun_out/ws/${v}_$d
    DXRL_WGRAD_DIAG=$d DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline > $o.log 2>&1 || exit 1
    f=$(ls $o/run_kernel_stats.csv $o/*/run_kernel_stats.csv 2>/dev/null | head -1)
    echo "$v diag=$d $(grep k_wgrad_l1 $f | awk -F, '{print $4/1000 " us"}')"
  done
done
