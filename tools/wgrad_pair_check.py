"""Gradients of one PG learner pass (rollout, critic values, advantages, both train passes) at
several sizes, saved to gpurun_out/wpc_<TAG>.pt, so two kernel libraries (DXRL_LIB) can be
compared bit for bit: python tools/wgrad_pair_check.py TAG  /  python tools/wgrad_pair_check.py
--compare TAG_A TAG_B.  The sizes give k_wgrad_l1 1, 2, 3, 5, 32, 33 and 100 chunks per
workgroup (odd counts and the short prologue included)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

SIZES = ((1, 32), (2, 32), (1, 96), (5, 32), (96, 64), (773, 32), (100, 32), (4096, 200))
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")

if sys.argv[1] == "--compare":
    a, b = (torch.load(os.path.join(OUT, f"wpc_{t}.pt"), weights_only=True) for t in sys.argv[2:4])
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print("bit-identical" if not bad else f"DIFFER at {bad}", flush=True)
    sys.exit(1 if bad else 0)

import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import envs, trainer  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for n, T in SIZES:
    env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named("easy"), reward_type="dense", seed=3, device=dev)
    tr = trainer.PGTrainer(env, trainer.TrainerConfig(horizon=T, seed=11))
    tr.rollout()
    for name in [x for x in tr.phases() if x not in ("rollout", "optimizer_step")]:
        getattr(tr, name)()
    torch.cuda.synchronize()
    res[f"{n}x{T}"] = tr.grads.detach().cpu().clone()
    print(n, T, "M", tr.M, "splits", tr.splits, "grad norm", round(tr.grads.double().norm().item(), 4), flush=True)
os.makedirs(OUT, exist_ok=True)
torch.save(res, os.path.join(OUT, f"wpc_{sys.argv[1]}.pt"))
