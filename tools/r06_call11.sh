#!/bin/bash
# round-6 GPU call 11: activation-fragment prefetch depth of fwd_pipe (DXRL_BD 3 / 4 / 5), kernel A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="C D E" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_bd.log 2>&1 || exit 4
cat gpurun_out/r06/abk_bd.log
