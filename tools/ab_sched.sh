# A/B of a compiler-flag variant of the whole library (EXTRA_FLAGS, tools/build_variant.py):
# GPU tests of the learner / rollout on the variant, rollout times and C2 / PPO bench lines,
# interleaved with the default build.  Libraries first (here):
#   EXTRA_FLAGS="-mllvm -amdgpu-sched-strategy=max-ilp" python tools/build_variant.py ilp
#   python tools/build_variant.py base;  then on the box: VARS="base ilp" bash tools/ab_sched.sh
set -o pipefail
O=gpurun_out/sched
mkdir -p $O
V=${VARS:-base ilp}
for v in $V; do [ "$v" = base ] && continue
  DXRL_LIB=ab/lib$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pg.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in $V; do
    DXRL_LIB=ab/lib$v.so CUR=easy timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
    DXRL_LIB=ab/lib$v.so timeout -k 10 120 python bench.py --config easy --no-cpu-baseline --no-roofline --steps 30 --warmup 3 > $O/b.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'C2', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['phases_ms'])" $O/b.log $v
  done
done
for v in $V; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 150 python bench.py --config easy --no-cpu-baseline --no-roofline --steps 15 --warmup 3 --epochs 4 --minibatches 4 > $O/b.log 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'PPO', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['phases_ms'])" $O/b.log $v
done
