"""A/B timing of one PG iteration's phases (rollout, critic values, actor / critic train) at the
bench shape (config_easy, 4096 envs x 200), HIP events, median of REPS repetitions per phase."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd  # noqa: E402,F401
from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

dev = torch.device("cuda:0")
kw = {"splitk_target_blocks": int(os.environ["SPLITK"])} if os.environ.get("SPLITK") else {}
env, tr = build_pg_workload(os.environ.get("CFG", "easy"), dev, **kw)
for _ in range(2):
    tr.iteration()
torch.cuda.synchronize()
reps = int(os.environ.get("REPS", "5"))
out = {}
for nm in ("rollout", "critic_values", "advantages", "actor_train", "critic_train", "optimizer_step"):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        getattr(tr, nm)()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    out[nm] = round(sorted(ts)[len(ts) // 2], 4)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    tr.iteration()
b.record()
torch.cuda.synchronize()
out["iteration"] = round(a.elapsed_time(b) / reps, 4)
print(os.environ.get("SPLITK", ""), out)
