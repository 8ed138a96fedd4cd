"""Learner kernels on two workloads' data in one process (alternating, HIP events): whether the
train passes' time depends on the data (C2 easy vs C5 variable + noise)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

dev = torch.device("cuda:0")
trs = {}
for name in ("easy", "variable_noise"):
    env, tr = build_pg_workload(name, dev)
    for _ in range(3):
        tr.iteration()
    tr.rollout()
    tr.critic_values()
    tr.advantages()
    trs[name] = tr
torch.cuda.synchronize()


def t(fn, reps=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for rnd in range(3):
    for name, tr in trs.items():
        print(rnd, name, {k: round(t(getattr(tr, k)), 4) for k in ("critic_values", "critic_train", "actor_train")},
              flush=True)
