# A/B of the dH2 store policy on one box: plain bench lines, then rocprofv3 kernel stats (C2)
# Libraries first: ab/libdh2nt.so and ab/libdh2plain.so as in tools/ab_dh2_bench.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ntprof
mkdir -p $O
line() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['value']/1e6,1), 'M', d['ms_per_step'], 'ms')" $1 $2; }
for r in 1 2; do
for v in dh2nt dh2plain; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 120 python bench.py --config easy --no-cpu-baseline --no-roofline --steps 30 --warmup 3 > $O/b_$v$r.log 2>&1 || exit 1
  line $O/b_$v$r.log "bench $v"
done
done
for v in dh2nt dh2plain; do
  DXRL_LIB=ab/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --config easy --no-cpu-baseline --no-roofline --steps 20 --warmup 3 > $O/p_$v.log 2>&1 || exit 1
  line $O/p_$v.log "rocprof $v"
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for row in csv.DictReader(open('$f')):
    n=row['Name']
    if any(k in n for k in ('k_wgrad_l1','k_pg_fused<8, 128, true','k_pg_rollout_ws','k_pg_fused<8, 128, false')):
        print('%9.1f us  %s' % (float(row['AverageNs'])/1e3, n[:60]))
"
done
