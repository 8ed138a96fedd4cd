#!/bin/bash
# round-6 evidence call: the GPU suite and the smoke at HEAD, then tools/profile_round.sh (ROUND=r06)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r/smoke.log 2>&1 || exit 5
tail -2 gpurun_out/r/smoke.log
ROUND=r06 bash tools/profile_round.sh
