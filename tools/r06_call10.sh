#!/bin/bash
# round-6 GPU call 10: GAE as a segmented wavefront scan (DXRL_GAE_SCAN): kernel == restatement
# tests, then the advantages-phase A/B (S = scan, Q = one chain per env), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py > gpurun_out/r06/pytest_gae_scan.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06/pytest_gae_scan.log; exit 3; }
tail -2 gpurun_out/r06/pytest_gae_scan.log
rm -f gpurun_out/ab.log
VARIANTS="S Q" bash tools/ab.sh 4 tools/adv_time.py > /dev/null 2>&1 || exit 4
cp gpurun_out/ab.log gpurun_out/r06/ab_gae_scan.log; cat gpurun_out/r06/ab_gae_scan.log
