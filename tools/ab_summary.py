"""Median per variant of an ab.log written by tools/ab.sh (bench.py JSON lines or the phase
tool's dict lines): python tools/ab_summary.py [gpurun_out/ab.log]"""
import ast
import collections
import json
import statistics
import sys

rows = collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    v, _, rest = line.strip().partition(" ")
    rest = rest.strip()
    if rest.startswith("{\""):
        d = json.loads(rest)
        rows[v].append({"ms_per_step": d["ms_per_step"], **d.get("phases_ms", {})})
    elif rest.startswith("{'"):
        rows[v].append(ast.literal_eval(rest))
for v, L in rows.items():
    keys = L[0].keys()
    print(f"{v:4s} n={len(L)}", {k: round(statistics.median(x[k] for x in L), 4) for k in keys})
