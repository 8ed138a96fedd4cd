#!/bin/bash
# round-6 GPU call 16: layer-2 activations stored by the rollout / critic-values pass and read by
# the first train pair (TrainerConfig.reuse_h2): tests, then the A/B (reuse vs --recompute-h2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r06/pytest_h2.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_h2.log; exit 3; }
tail -2 gpurun_out/r06/pytest_h2.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
for i in 1 2 3; do
  for v in reuse recompute; do
    extra=""; [ $v = recompute ] && extra="--recompute-h2"
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $extra > gpurun_out/abk/${v}_$i.log 2>&1 || exit 4
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/r06/abk_h2.log 2>&1
cat gpurun_out/r06/abk_h2.log
