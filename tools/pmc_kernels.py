"""Per-kernel summary of rocprofv3 --pmc counter CSVs (any counters), with the MFMA view:

    python tools/pmc_kernels.py "<glob of *counter_collection.csv>" [kernel substrings ...]

For each kernel (name prefix) and counter: dispatches, mean value per dispatch.  When
SQ_INSTS_VALU_MFMA_MOPS_BF16 is present, FLOP per dispatch = 512 x MOPS (the unit of
the MOPS counters) is printed beside it, and SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE
are reported as collected (GRBM_GUI_ACTIVE is summed over the 8 XCDs)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(pattern):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "").split("(")[0]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main(pattern, keys):
    acc = load(pattern)
    out = {}
    for name, ctrs in sorted(acc.items()):
        if keys and not any(k in name for k in keys):
            continue
        d = {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in ctrs.items()}
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in d:
            d["mfma_bf16_flop_per_dispatch"] = 512.0 * d["SQ_INSTS_VALU_MFMA_MOPS_BF16"]["mean"]
        out[name[:80]] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
