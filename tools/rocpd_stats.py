"""Per-kernel duration stats (calls, average / min µs) from a rocprofv3 rocpd database (run_results.db),
for runs recorded without --output-format csv.  usage: python tools/rocpd_stats.py <db> [top]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
names = dict(c.execute("select id, display_name from rocpd_info_kernel_symbol"))
d = collections.defaultdict(list)
for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
    d[names.get(kid, str(kid))].append((e - s) / 1e3)
rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]
for n, v in rows:
    print(f"{len(v):6d} {sum(v) / len(v):10.2f} us avg {min(v):9.2f} min  {n[:90]}")
