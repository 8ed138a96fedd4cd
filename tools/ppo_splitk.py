"""PPO 4 x 4 iteration time vs the dW2 split-K block target (A/B of the per-pass partial traffic):
    python tools/ppo_splitk.py 768 384 192"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

dev = torch.device("cuda:0")
for rep in range(2):
    for sk in [int(a) for a in sys.argv[1:]]:
        env, tr = build_pg_workload("easy", dev, epochs=4, minibatches=4, splitk_target_blocks=sk)
        for _ in range(2):
            tr.iteration()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(8):
            tr.iteration()
        b.record()
        torch.cuda.synchronize()
        print(f"splitk_target_blocks={sk} splits={tr.splits} ms_per_iteration={a.elapsed_time(b) / 8:.3f}", flush=True)
        del env, tr
        torch.cuda.empty_cache()
