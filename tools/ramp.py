"""Per-iteration GPU time of the bench workload from a cold start (HIP events around each
iteration): shows how many iterations the clocks take to reach steady state."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

dev = torch.device("cuda:0")
env, tr = build_pg_workload(os.environ.get("CFG", "easy"), dev)
n = int(os.environ.get("ITERS", "40"))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
t0 = time.perf_counter()
ev[0].record()
for k in range(n):
    tr.iteration()
    ev[k + 1].record()
torch.cuda.synchronize()
print("host enqueue+run s", round(time.perf_counter() - t0, 3))
print(" ".join(f"{ev[k].elapsed_time(ev[k + 1]):.3f}" for k in range(n)))
