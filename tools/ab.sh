#!/bin/bash
# A/B two library builds on one box: ab/libA.so vs ab/libB.so, alternating, N rounds.
# usage: bash tools/ab.sh [rounds] [script]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-3}
S=${2:-tools/fused_bench.py}
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in A B; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 120 python "$S" 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/ab.log || exit 1
  done
done
