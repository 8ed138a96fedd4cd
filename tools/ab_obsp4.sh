# A/B of DXRL_WS_OBS_IN_P4 (k_pg_rollout_ws writes observation row t + 1 at the end of step t's
# P4; no P0 phase).  Libraries first (here): printf '#define DXRL_WS_OBS_IN_P4 0' > o;
#   printf '#define DXRL_WS_OBS_IN_P4 1' > n; python tools/build_variant.py obsp4 dxrl_pg.hip o n;
#   python tools/build_variant.py base
set -o pipefail
O=gpurun_out/obsp4
mkdir -p $O
DXRL_LIB=ab/libobsp4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pg.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "obsp4 $(tail -1 $O/pytest.log)"
for r in 1 2 3; do
  for v in base obsp4; do
    for c in easy variable; do
      DXRL_LIB=ab/lib$v.so CUR=$c timeout -k 10 120 python tools/rollout_time.py 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
    done
  done
done
for r in 1 2; do
  for v in base obsp4; do
    DXRL_LIB=ab/lib$v.so timeout -k 10 120 python bench.py --config easy --no-cpu-baseline --no-roofline --steps 30 --warmup 3 > $O/b.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'C2', round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['phases_ms'])" $O/b.log $v
  done
done
