set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ws2
for sk in 384 768 1536; do
  for d in 3 0; do
    o=gpurun_out/ws2/s${sk}_$d
    SPLITK=$sk DXRL_WGRAD_DIAG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- python3 tools/wgrad_splits.py > $o.log 2>&1 || exit 1
    f=$(ls $o/run_kernel_stats.csv $o/*/run_kernel_stats.csv 2>/dev/null | head -1)
    echo "splitk=$sk diag=$d $(grep k_wgrad_l1 $f | awk -F, '{print $4/1000 " us"}') $(grep splits $o.log)"
  done
done
