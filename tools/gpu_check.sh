#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel stats.
# Stops at the first step that faults / aborts / times out (exit 124,134,137,139).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" | tee -a $OUT/session.log
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "fatal exit $rc in $name; stopping" | tee -a $OUT/session.log; exit $rc; fi
  return 0
}
STEPS=${STEPS:-pytest smoke bench prof}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    configs) for c in default hard_heldout variable_noise; do
               run bench_$c 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-roofline
             done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
  esac
done
