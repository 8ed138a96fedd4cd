"""Time the advantages phase (GAE + moments) at the bench shape with HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

dev = torch.device("cuda:0")
env = envs.VecEnv(4096, curriculum_config=pkg.CurriculumConfig.named("easy"), reward_type="dense", seed=1, device=dev)
tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=200, seed=7))
env.reset(write_obs=False)
tr.rollout()
tr.critic_values()
tr.advantages()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50):
    tr.advantages()
b.record()
torch.cuda.synchronize()
print("advantages ms", round(a.elapsed_time(b) / 50, 4), "stats", [round(float(x), 6) for x in tr.stats[:5].cpu()])
