#!/bin/bash
# round-6 GPU call 15: slab sums with 16 loads in flight (DXRL_SLAB_B16)
# (X = 8 as before, Y = 16 in-tree): learner tests on the in-tree build, then the
# kernel A/B over C2 and over PPO 4 x 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_gpu_rccl.py > gpurun_out/r06/pytest_slab_b16.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_slab_b16.log; exit 3; }
tail -2 gpurun_out/r06/pytest_slab_b16.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="X Y" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_slab_b16.log 2>&1 || exit 4
cat gpurun_out/r06/abk_slab_b16.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="X Y" bash tools/ab_kernels.sh 2 --epochs 4 --minibatches 4 --steps 8 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/r06/abk_slab_b16_ppo.log 2>&1 || exit 5
cat gpurun_out/r06/abk_slab_b16_ppo.log
