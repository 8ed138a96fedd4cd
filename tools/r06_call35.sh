#!/bin/bash
# the 32-env rollout kernel writes the actor's layer-2 tape too: parity (stored-H2 and rollout
# tests, the 8192-env cases on the 32-env kernel), then C4 iteration time tape / notape interleaved
# and C4 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py > gpurun_out/r06/pytest_e8tape.log 2>&1 || { tail -30 gpurun_out/r06/pytest_e8tape.log; exit 1; }
tail -1 gpurun_out/r06/pytest_e8tape.log
for i in 1 2 3; do for v in notape tape; do
  VARIANT=$v timeout -k 10 150 python tools/e8_tape_ab.py 2>&1 | grep -v amdgpu >> gpurun_out/r06/e8_tape_ab.log || exit 2
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --config hard_heldout --no-cpu-baseline --no-roofline > gpurun_out/r06/bench_c4_e8tape.log 2>&1 || exit 3
grep '^{' gpurun_out/r06/bench_c4_e8tape.log | cut -c1-200
python3 tools/trace_summary.py gpurun_out/prof_c4/run_kernel_trace.csv | head -8
cat gpurun_out/r06/e8_tape_ab.log
