"""Time the standalone step kernel (dxrl_env_step) at a large N: bytes / HIP-event time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs  # noqa: E402

n = int(os.environ.get("ENVS", str(1 << 22)))
dev = torch.device("cuda:0")
env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.variable(), reward_type="dense", seed=5, device=dev)
env.reset(write_obs=False)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = (torch.rand(n, 15, generator=g, device=dev) * 2.4 - 1.2).contiguous()
for _ in range(3):
    env.step(acts)
torch.cuda.synchronize()
L = 30
variants = os.environ.get("VARIANTS", "default").split(",")
res = {v: [] for v in variants}
for rep in range(int(os.environ.get("REPS", "1"))):
    for v in variants:
        if v == "default":
            os.environ.pop("DXRL_STEP_VARIANT", None)
        else:
            os.environ["DXRL_STEP_VARIANT"] = v
        env.step(acts)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(L + 1)]
        ev[0].record()
        for k in range(L):
            env.step(acts)
            ev[k + 1].record()
        torch.cuda.synchronize()
        res[v].append(sum(ev[k].elapsed_time(ev[k + 1]) for k in range(L)) / L)
for v in variants:
    ms = sorted(res[v])[len(res[v]) // 2]
    print(f"variant={v} envs={n} median ms={ms:.4f} GB/s={594 * n / (ms * 1e-3) / 1e9:.1f} "
          f"all={[round(x, 4) for x in res[v]]}")
