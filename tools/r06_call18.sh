#!/bin/bash
# round-6 GPU call 18: stored H2 variants at the bench shape -- the critic-values pass's H2 store
# non-temporal (N, in-tree) or plain (B, commit b1ff78b); actor tape + critic H2 (both), actor only,
# neither (none) -- interleaved x3 (tools/h2_ab.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pg.py -k "h2 or values or iteration" > gpurun_out/r06/pytest_h2_nt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06/pytest_h2_nt.log; exit 3; }
tail -2 gpurun_out/r06/pytest_h2_nt.log
rm -f gpurun_out/r06/ab_h2_variants.log
for i in 1 2 3; do
  for lv in "N both" "B both" "N actor" "N none"; do
    set -- $lv
    DXRL_LIB=ab/lib$1.so VARIANT=$2 timeout -k 10 120 python tools/h2_ab.py 2>&1 | grep -v amdgpu | sed "s/^/$1 /" >> gpurun_out/r06/ab_h2_variants.log || exit 4
  done
done
cat gpurun_out/r06/ab_h2_variants.log
