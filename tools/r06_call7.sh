#!/bin/bash
# round-6 GPU call 7: LDS-wait fixes (gate preload, batched db2 reads, copy-out schedule) A/B, then
# the learner tests on the in-tree build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="I V" bash tools/ab_kernels.sh 4 > gpurun_out/r06/abk_ldswait.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py > gpurun_out/r06/pytest_call7.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/r06/pytest_call7.log
