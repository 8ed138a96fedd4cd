#!/bin/bash
# round-6 GPU call 5: weight prefetch depth / packed dH2 gate, kernel-level A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="I P Q R U" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_wpf_gatepk.log 2>&1 || exit 3
echo done
