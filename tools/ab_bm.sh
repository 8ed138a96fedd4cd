# A/B of the Box-Muller implementation (hardware log2 / sin / cos in revolutions vs __logf /
# __sincosf): GPU tests on the new library, rollout-time ratios (C2 easy, C5 variable + noise,
# C4 hard at 8192 envs) and C2 / C5 bench lines, interleaved on one box
# Libraries first: SRC_REV=<commit before the change> python tools/build_variant.py bmold;
#   python tools/build_variant.py bmnew
set -o pipefail
O=gpurun_out/bm
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_pg.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2 3; do
  for v in bmold bmnew; do
    for c in easy variable; do
      DXRL_LIB=ab/lib$v.so CUR=$c timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
    done
    DXRL_LIB=ab/lib$v.so CUR=hard ENVS=8192 timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v 8192 /" || exit 1
  done
done
for r in 1 2; do
  for v in bmold bmnew; do
    for c in easy variable_noise; do
      DXRL_LIB=ab/lib$v.so timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-roofline --steps 30 --warmup 3 > $O/b.log 2>&1 || exit 1
      python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms rollout', d['phases_ms']['rollout'])" $O/b.log $v $c
    done
  done
done
