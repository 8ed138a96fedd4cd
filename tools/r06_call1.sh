#!/bin/bash
# round-6 GPU call: changed tests, learner early-weight A/B, C5 noise rollout A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bench_harness.py tests/test_gpu_pg.py tests/test_gpu_fullsize.py \
  "tests/test_gpu_parity.py::test_streaming_step_policy_is_bit_identical" > gpurun_out/r06/pytest_call1.log 2>&1
rc=$?; echo "pytest rc=$rc"; ok $rc || exit $rc
rm -f gpurun_out/ab.log
VARIANTS="A B E F G" bash tools/ab.sh 3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > /dev/null 2>&1 || exit 3
mv gpurun_out/ab.log gpurun_out/r06/ab_early_w.log
for i in 1 2 3; do for v in A B; do for c in easy variable; do
  DXRL_LIB=ab/lib$v.so CUR=$c DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/rollout_noise_ab.log || exit 4
done; done; done
echo done
