"""Throughput of the device evaluation programs (k_eval): held-out evaluation,
parallel form with device Philox streams.  Prints one JSON line per workload."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import dexterous_rl_manipulation_amd as pkg  # noqa: E402
from dexterous_rl_manipulation_amd import evaluation as ev, evaluator as evr  # noqa: E402

MEAN = [-0.3, -0.2, -0.1, 0.1, 0.2, 0.3, -0.4, -0.4, 0.0, 0.25, -0.25, 0.1, -0.1, 0.05, -0.05]


class Frozen:
    exploration_noise = 0.3
    mean_action = np.asarray(MEAN, np.float32)


def measured_efficiency(p, prog, steps, hist):
    """One diagnostic launch (DXRL_EVAL_DIAG=1): the kernel reports the step iterations its waves
    executed; each iteration of a 64-lane wave offers 4 env-step slots (k_eval_ls: 16 lanes per
    env) or 64 (the one-lane kernel).  Efficiency = env steps / slots."""
    import os
    import tempfile
    one = os.environ.get("DXRL_EVAL_ONE_LANE", "0") not in ("", "0")
    if one:
        return None
    os.environ["DXRL_EVAL_DIAG"] = "1"
    with tempfile.TemporaryFile(mode="w+") as f:
        saved = os.dup(2)
        os.dup2(f.fileno(), 2)
        try:
            p.run(prog, host_resets=False, host_noise=False, keep_history=hist)
        finally:
            os.dup2(saved, 2)
            os.close(saved)
            del os.environ["DXRL_EVAL_DIAG"]
        f.seek(0)
        line = [x for x in f.read().splitlines() if "wave_iterations=" in x][-1]
    it = int(line.split("wave_iterations=")[1].split()[0])
    return steps / (4 * it)


def wave_steps(lengths):
    """Lane-steps the waves execute: every lane of a 64-lane wave runs as long as its longest episode."""
    L = np.zeros(-(-len(lengths) // 64) * 64, np.int64)
    L[:len(lengths)] = lengths
    return int(L.reshape(-1, 64).max(1).sum() * 64)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    hist = len(sys.argv) > 2 and sys.argv[2] == "hist"
    for cfg in ("hard", "variable"):
        h = ev.HeldOutObjectSet(getattr(pkg.CurriculumConfig, cfg)(), num_heldout_objects=10, seed=42)
        e = ev.Evaluator(Frozen(), h, max_episode_steps=200)
        prog = evr.policy_program(e.policy)
        p = e.heldout_program(K, 0, parallel=True)
        t = {}
        p.run(prog, host_resets=False, host_noise=False, keep_history=hist)  # warm
        t0 = time.perf_counter()
        rec = p.run(prog, host_resets=False, host_noise=False, keep_history=hist, repeat=20, timing=t)
        wall = time.perf_counter() - t0
        steps = int(rec.ep_length.astype(np.int64).sum())
        E = len(rec.ep_length)
        print(json.dumps({"workload": f"heldout {cfg} 10 objects x {K} episodes, frozen SimpleLearner, dense",
                          "episodes": E, "env_steps": steps, "mean_length": steps / E,
                          "kernel_ms": round(t["kernel_ms"], 4), "episodes_per_s": E / (t["kernel_ms"] * 1e-3),
                          "env_steps_per_s": steps / (t["kernel_ms"] * 1e-3),
                          "wave_efficiency_one_lane_model": steps / wave_steps(rec.ep_length),
                          "wave_efficiency_measured": measured_efficiency(p, prog, steps, hist),
                          "success_rate": float(rec.ep_success.mean()), "host_wall_s_20_launches": wall}))


if __name__ == "__main__":
    main()
