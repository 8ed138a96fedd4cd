"""Time the learner phases (fused or GEMM chain) at the bench shape with HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

n = int(os.environ.get("ENVS", "4096"))
dev = torch.device("cuda:0")
env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named("hard"), reward_type="dense", seed=1, device=dev)
tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=200, seed=7))
env.reset(write_obs=False)
tr.rollout()
tr.critic_values()
tr.advantages()
names = ["critic_values", "actor_train", "critic_train"]
for nm in names:
    getattr(tr, nm)()
torch.cuda.synchronize()
reps = 5
out = {}
for nm in names:
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        getattr(tr, nm)()
    b.record()
    torch.cuda.synchronize()
    out[nm] = round(a.elapsed_time(b) / reps, 4)
print(os.environ.get("DXRL_FUSED_TILE", "128"), out, tr.loss_stats())
