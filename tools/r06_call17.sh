#!/bin/bash
# round-6 GPU call 17: the critic-values pass's H2 copy spread over the next tile's layer-1 steps
# (S, in-tree) vs a burst after the barrier (B, commit b1ff78b): tests, then the kernel A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "h2 or values or iteration" > gpurun_out/r06/pytest_h2_spread.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_h2_spread.log; exit 3; }
tail -2 gpurun_out/r06/pytest_h2_spread.log
rm -rf gpurun_out/abk; mkdir -p gpurun_out/abk
VARIANTS="B S" bash tools/ab_kernels.sh 3 > gpurun_out/r06/abk_h2_spread.log 2>&1 || exit 4
cat gpurun_out/r06/abk_h2_spread.log
for v in B S; do DXRL_LIB=ab/lib$v.so timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,1), d['ms_per_step'], d['phases_ms'])"; done
