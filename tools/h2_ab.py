"""A/B of the stored layer-2 activations at the bench shape (config_easy, 4096 x 200, 1 x 1):
VARIANT=both (actor tape + critic H2), actor (actor tape only), none (recompute both).
Prints ms per iteration (HIP events over 20 iterations after a 2 s prewarm) and the phases."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

v = os.environ.get("VARIANT", "both")
dev = torch.device("cuda:0")
env, tr = build_pg_workload("easy", dev, envs=4096, horizon=200, reuse_h2=v != "none")
if v == "actor":
    tr.h2c = None
t0 = time.time()
while time.time() - t0 < 2.0:
    tr.iteration()
    torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    tr.iteration()
b.record()
torch.cuda.synchronize()
print(v, "ms/iter", round(a.elapsed_time(b) / 20, 4))
