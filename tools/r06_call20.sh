#!/bin/bash
# H2 DMA skew A/B: iteration time (tools/h2_ab.py) over libh2A (no skew) .. libh2D, interleaved,
# then per-kernel durations (rocprofv3 over bench.py) for A vs C
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abk
VARIANTS="h2A h2B h2C h2D" bash tools/ab.sh 3 tools/h2_ab.py || exit 1
VARIANTS="h2A h2C h2D" bash tools/ab_kernels.sh 2 > gpurun_out/abk_summary.log 2>&1 || exit 2
cat gpurun_out/abk_summary.log
for i in 1 2; do timeout -k 10 200 python bench.py --epochs 4 --minibatches 4 --steps 10 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/ppo_$i.log 2>&1 || exit 3; grep '^{' gpurun_out/ppo_$i.log | cut -c1-200; done
