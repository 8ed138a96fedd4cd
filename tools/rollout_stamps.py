"""Per-step segment cycles of k_pg_rollout_ls (diag flag 32; diagnostic only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

for cur in ("easy", "hard"):
    env = envs.VecEnv(4096, curriculum_config=pkg.CurriculumConfig.named(cur), reward_type="dense", seed=1,
                      device=torch.device("cuda:0"))
    tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=200, seed=7))
    env.reset(write_obs=False)
    tr.rollout()
    tr.diag_flags = int(os.environ.get("DIAG", "128"))
    print(cur, flush=True)
    tr.rollout()
    torch.cuda.synchronize()
