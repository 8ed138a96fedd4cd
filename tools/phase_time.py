"""Time trainer phases at a bench shape after a clock prewarm (HIP events, back-to-back calls):
PHASES (default critic_values) x REPS, ROUNDS rounds; CONFIG workload (default easy).
Run under tools/ab.sh to compare library builds on one box."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

dev = torch.device("cuda:0")
env, tr = build_pg_workload(os.environ.get("CONFIG", "easy"), dev)
phases = os.environ.get("PHASES", "critic_values").split(",")
reps, rounds = int(os.environ.get("REPS", "40")), int(os.environ.get("ROUNDS", "3"))
t0 = time.time()
while time.time() - t0 < float(os.environ.get("PREWARM_S", "2")):
    tr.iteration()
tr.rollout()
tr.critic_values()
tr.advantages()
torch.cuda.synchronize()
out = {}
for _ in range(rounds):
    for ph in phases:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            getattr(tr, ph)()
        b.record()
        torch.cuda.synchronize()
        out.setdefault(ph, []).append(round(a.elapsed_time(b) / reps * 1e3, 1))
print({k: v for k, v in out.items()}, "us", float(tr.V[0, :4096].double().sum()))
