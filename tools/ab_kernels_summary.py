"""Median over rounds of each kernel's average duration (us) per variant, from tools/ab_kernels.sh."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abk"
data = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, "*", "**", "*kernel_stats.csv"), recursive=True):
    v = os.path.relpath(path, root).split(os.sep)[0].rsplit("_", 1)[0]
    for row in csv.DictReader(open(path)):
        name = row["Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        data[name][v].append(float(row["AverageNs"]) / 1000.0)
variants = sorted({v for d in data.values() for v in d})
tot = {n: max(statistics.median(x) for x in d.values()) for n, d in data.items()}
print("kernel".ljust(62), " ".join(v.rjust(9) for v in variants))
for n in sorted(data, key=lambda n: -tot[n])[:14]:
    print(n.ljust(62), " ".join((f"{statistics.median(data[n][v]):9.1f}" if v in data[n] else " " * 9) for v in variants))

# Clock-normalised view: box clock drifts between runs by a few per cent (DVFS), so each run's
# averages are also divided by an unchanged reference kernel of the SAME run (AB_REF, default the
# rollout), then multiplied by that kernel's median over all runs.
ref = os.environ.get("AB_REF", "k_pg_rollout_ws")
runs = collections.defaultdict(dict)  # (variant, run dir) -> kernel -> us
for path in glob.glob(os.path.join(root, "*", "**", "*kernel_stats.csv"), recursive=True):
    run = os.path.relpath(path, root).split(os.sep)[0]
    for row in csv.DictReader(open(path)):
        name = row["Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        runs[run][name] = float(row["AverageNs"]) / 1000.0
refname = next((n for n in data if ref in n), None)
if refname:
    base = statistics.median(r[refname] for r in runs.values() if refname in r)
    norm = collections.defaultdict(lambda: collections.defaultdict(list))
    for run, ks in runs.items():
        if refname not in ks:
            continue
        v = run.rsplit("_", 1)[0]
        for n, us in ks.items():
            norm[n][v].append(us * base / ks[refname])
    print(f"\nnormalised to {refname.strip()} (median {base:.1f} us) per run:")
    for n in sorted(data, key=lambda n: -tot[n])[:8]:
        print(n.ljust(62), " ".join((f"{statistics.median(norm[n][v]):9.1f}" if v in norm[n] else " " * 9) for v in variants))
