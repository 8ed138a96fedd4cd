"""Run a few PG iterations (config_easy, 4096 envs, T=200) for rocprofv3 kernel traces."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

n = int(os.environ.get("PROF_ENVS", "4096"))
T = int(os.environ.get("PROF_T", "200"))
iters = int(os.environ.get("PROF_ITERS", "3"))
dev = torch.device("cuda:0")
env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.easy(), reward_type="dense", seed=1, device=dev)
ep, mb = int(os.environ.get("PROF_EPOCHS", "1")), int(os.environ.get("PROF_MB", "1"))
tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=T, seed=7, epochs=ep, minibatches=mb))
env.reset(write_obs=False)
for _ in range(iters):
    tr.iteration()
torch.cuda.synchronize()
print("ok")
