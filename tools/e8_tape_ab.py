"""C4 (hard + held-out, 8192 envs: the 32-env rollout kernel) iteration time with the actor's
layer-2 tape written by the 32-env kernel (VARIANT=tape) or not (VARIANT=notape: the actor's
first train pass recomputes layer 2). HIP events over 10 iterations after a 2 s prewarm."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd import trainer as T  # noqa: E402
from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

v = os.environ.get("VARIANT", "tape")
if v == "notape":
    T.TAPE_KERNELS = (1,)
env, tr = build_pg_workload("hard_heldout", torch.device("cuda:0"), envs=8192, horizon=200)
t0 = time.time()
while time.time() - t0 < 2.0:
    tr.iteration()
    torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    tr.iteration()
b.record()
torch.cuda.synchronize()
print(v, "tape_written", tr.h2a_tape_written, "ms/iter", round(a.elapsed_time(b) / 10, 4))
