#!/bin/bash
# A/B library builds on one box (tools/build_variant.py -> ab/lib<V>.so), interleaved, N rounds.
# usage: VARIANTS="A B C" bash tools/ab.sh [rounds] [script args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-3}
shift || true
S=${*:-tools/fused_bench.py}
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in ${VARIANTS:-A B}; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 120 python $S 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 1
  done
done
cat gpurun_out/ab.log
