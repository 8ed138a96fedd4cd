"""Run the critic train pass (fused pass + k_wgrad_l1 + reduction) at the bench shape with
SPLITK=<splitk_target_blocks> (wgrad splits = SPLITK // 3), for rocprofv3 kernel stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

dev = torch.device("cuda:0")
env = envs.VecEnv(4096, curriculum_config=pkg.CurriculumConfig.named("easy"), reward_type="dense", seed=1, device=dev)
tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=200, seed=7,
                                                  splitk_target_blocks=int(os.environ.get("SPLITK", "768"))))
env.reset(write_obs=False)
tr.rollout()
tr.critic_values()
tr.advantages()
for _ in range(6):
    tr.critic_train()
torch.cuda.synchronize()
print("splits", tr.splits)
