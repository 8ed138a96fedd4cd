#!/bin/bash
# round-6 GPU call 4: the whole GPU suite, smoke and one bench line at the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06/pytest_gpu_full.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || exit 5
timeout -k 10 300 python bench.py > gpurun_out/r06/bench_easy_call4.json 2> gpurun_out/r06/bench_easy_call4.err || exit 6
echo done
