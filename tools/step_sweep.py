"""k_step roofline sweep: N = 2^12 .. 2^24 envs, HIP events over
back-to-back launches, 594 algorithmic bytes per env-step.  One JSON line per N.

    python tools/step_sweep.py [lo_exp] [hi_exp] > profiles/rNN/step_sweep.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

lo, hi = (int(sys.argv[1]) if len(sys.argv) > 1 else 12), (int(sys.argv[2]) if len(sys.argv) > 2 else 24)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for e in range(lo, hi + 1):
    n = 1 << e
    launches = max(20, min(400, (1 << 26) // n))
    ms = bench.step_kernel_time(n, launches, dev)
    gbs = bench.STEP_BYTES_PER_ENV * n / (ms * 1e-3) / 1e9
    print(json.dumps({"envs": n, "log2": e, "launches": launches, "us_per_launch": round(ms * 1e3, 3),
                      "env_steps_per_s": round(n / (ms * 1e-3), 1), "algorithmic_GB_s": round(gbs, 1),
                      "frac_of_8TBs": round(gbs / bench.PEAK_HBM_GBS, 4),
                      "traffic_over_infinity_cache": bench.STEP_BYTES_PER_ENV * n > 256 * 2**20}), flush=True)
