"""Per-dispatch summary of a rocprofv3 kernel trace: kernel, grid, avg/total us (last iteration order)."""
import csv
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = OrderedDict()
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
for (name, gx, gy, gz), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / c:10.1f} us x{c:4d} {100 * t / tot:5.1f}%  grid=({gx},{gy},{gz})  {name}")
