"""Time the fused PG rollout kernels (the default selection; ONE=1 adds the one-lane-per-env
kernel, diag 16; DIAGS=flags:name,... picks them, e.g. 0:default,2048:ws16,1024:e8) at the bench
shape (ENVS, default 4096; CUR the curriculum preset), one line."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

dev = torch.device("cuda:0")
cur = os.environ.get("CUR", "easy")
out = []
for noise in (0.0, 0.05):
    env = envs.VecEnv(int(os.environ.get("ENVS", "4096")), curriculum_config=pkg.CurriculumConfig.named(cur), reward_type="dense", seed=1, device=dev)
    tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=200, seed=7, obs_noise_std=noise, dyn_noise_std=noise))
    env.reset(write_obs=False)
    kernels = ((0, "default"),) + (((16, "one"),) if os.environ.get("ONE") else ())
    if os.environ.get("DIAGS"):  # e.g. DIAGS=0:default,2048:ws16,1024:e8
        kernels = tuple((int(d.split(":")[0]), d.split(":")[1]) for d in os.environ["DIAGS"].split(","))
    for flags, name in kernels:
        tr.diag_flags = flags
        tr.rollout()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            tr.rollout()
        b.record()
        torch.cuda.synchronize()
        out.append(f"{name}{'+noise' if noise else ''}={a.elapsed_time(b) / 10:.3f}")
print(cur, " ".join(out))
