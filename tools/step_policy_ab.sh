#!/bin/bash
# k_step cache-policy A/B per batch size: variants 0 plain, 1 nt stores,
# 2 nt loads, 3 both; interleaved REPS rounds per N on one box (tools/step_bench.py).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for e in ${EXPS:-17 18 19 20 21 22}; do
  ENVS=$((1 << e)) VARIANTS=${VARIANTS:-0,1,2,3} REPS=${REPS:-7} timeout -k 10 180 python tools/step_bench.py
done
