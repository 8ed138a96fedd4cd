#!/bin/bash
# Kernel-level A/B: rocprofv3 --kernel-trace --stats over bench.py for each variant library
# (ab/lib<V>.so), interleaved, N rounds; per-kernel average durations in gpurun_out/abk/<V>_<i>/.
#   VARIANTS="A B" bash tools/ab_kernels.sh [rounds] [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
N=${1:-2}
shift || true
ARGS=${*:---steps 20 --warmup 3 --no-cpu-baseline --no-roofline}
for i in $(seq 1 "$N"); do
  for v in ${VARIANTS:-A B}; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py $ARGS > gpurun_out/abk/${v}_$i.log 2>&1 || exit 1
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk
