set -o pipefail
for r in 1 2 3; do for pw in 1 2 3; do
timeout -k 10 120 python bench.py --config easy --no-cpu-baseline --no-roofline --prewarm-s $pw > gpurun_out/pw.log 2>&1 || exit 1
python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/pw.log') if l.startswith('{')][-1])
print('prewarm', sys.argv[1], round(d['value']/1e6,1), 'M', d['ms_per_step'], d['train_stats']['prewarm'])" $pw
done; done
