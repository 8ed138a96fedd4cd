# A/B of the dH2 store policy on one box: bench lines only (C2), three interleaved rounds
# Libraries first (here): printf '#define DXRL_DH2_NT 0' > o; printf '#define DXRL_DH2_NT 1' > n;
#   python tools/build_variant.py dh2nt dxrl_pg_fused.hip o n; python tools/build_variant.py dh2plain
#   then on the box: VARS="dh2plain dh2nt" bash tools/ab_dh2_bench.sh (VARS: any ab/lib<V>.so names)
set -o pipefail
O=gpurun_out/ntb
mkdir -p $O
for r in 1 2 3; do
for v in ${VARS:-dh2nt dh2plain}; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 120 python bench.py --config easy --no-cpu-baseline --no-roofline --steps 30 --warmup 3 > $O/b_$v$r.log 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms', d['phases_ms'])" $O/b_$v$r.log $v
done
done
