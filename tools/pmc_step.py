"""Drive k_step (dxrl_env_step) at a fixed large N for PMC collection.
Run under: rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -- python3 tools/pmc_step.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs  # noqa: E402

n = int(os.environ.get("PMC_ENVS", str(1 << 22)))
launches = int(os.environ.get("PMC_LAUNCHES", "8"))
dev = torch.device("cuda:0")
env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.variable(), reward_type="dense", seed=5, device=dev)
env.reset(write_obs=False)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = (torch.rand(n, 15, generator=g, device=dev) * 2.4 - 1.2).contiguous()
for _ in range(launches):
    env.step(acts)
torch.cuda.synchronize()
print("ok", n, launches)
