"""Restatement / reference speed ratio on one core, build container only.

    cd /tmp && python3 -B /root/repo/tools/cpu_ratio.py [seconds] [curriculum]

Times the reference's own loop (envs.DexterousManipulationEnv + SimpleLearner through
training/episode_utils.run_episode, imported read-only from /root/reference with the
tests/golden/gen_golden.py gymnasium stand-in) and bench.py's CPU-baseline loop over the
oracle restatement, same curriculum, same core, `seconds` each.  The reference never
travels to the GPU box; the ratio lets the box's oracle figure be read in reference units."""
import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def reference_rate(seconds, curriculum):
    import gen_golden
    gen_golden.install_gym_standin()
    sys.path.insert(0, gen_golden.REF)
    from envs.manipulation_env import DexterousManipulationEnv
    from experiments.config import CurriculumConfig
    from policies.simple_learner import SimpleLearner
    from training.episode_utils import run_episode
    cur = getattr(CurriculumConfig, curriculum)() if hasattr(CurriculumConfig, curriculum) else CurriculumConfig()
    env = DexterousManipulationEnv(reward_type="dense", curriculum_config=cur)
    np.random.seed(42)
    pol = SimpleLearner(env.action_space, learning_rate=0.01)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, n, _ = run_episode(env, pol, max_steps=200)
        steps += n
    return steps / (time.perf_counter() - t0)


def oracle_rate(seconds, curriculum):
    import queue
    import bench
    q = queue.Queue()
    bench._cpu_worker(curriculum, seconds, 0, q)
    steps, dt = q.get()
    return steps / dt


if __name__ == "__main__":
    sec = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    cur = sys.argv[2] if len(sys.argv) > 2 else "easy"
    r = reference_rate(sec, cur)
    o = oracle_rate(sec, cur)
    print(f"curriculum={cur} reference={r:.1f} env-steps/s oracle={o:.1f} env-steps/s ratio={o / r:.2f}")
