#!/bin/bash
# the actor's H2 tape copied by the aux waves in their P4 slack (TA1) vs by the env waves in the head
# phase (TA0): tape / stored-H2 parity on TA1, rollout stamps and interleaved rollout times of both,
# kernel A/B with rotated order
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06 gpurun_out/abk
DXRL_LIB=ab/libTA1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pg.py tests/test_gpu_fullsize.py > gpurun_out/r06/pytest_TA1.log 2>&1 || { tail -30 gpurun_out/r06/pytest_TA1.log; exit 1; }
tail -1 gpurun_out/r06/pytest_TA1.log
for v in TA0 TA1; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 120 python tools/rollout_stamps.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/ta_stamps.log || exit 2
done
for i in 1 2 3; do for v in TA0 TA1 ; do
  DXRL_LIB=ab/lib$v.so CUR=easy DIAGS=0:ws timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> gpurun_out/r06/ta_rt.log || exit 3
done; done
i=0
for order in "TA0 TA1" "TA1 TA0" "TA0 TA1" "TA1 TA0"; do
  i=$((i+1))
  for v in $order; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/${v}_$i -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/abk/${v}_$i.log 2>&1 || exit 4
    grep '^{' gpurun_out/abk/${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"]/1e6,1), d["ms_per_step"])' >> gpurun_out/r06/ta_bench.log
  done
done
python3 tools/ab_kernels_summary.py gpurun_out/abk > gpurun_out/abk_summary.log
cat gpurun_out/r06/ta_stamps.log gpurun_out/r06/ta_rt.log gpurun_out/r06/ta_bench.log gpurun_out/abk_summary.log
