"""Loaders for the committed golden fixtures (tests/golden/, made by gen_golden.py)."""
import functools
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(None)
def meta():
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        return json.load(f)


@functools.lru_cache(None)
def npz(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def env_case(i):
    z = npz("env_traces")
    pre = f"c{i}_"
    return {k[len(pre):]: v for k, v in z.items() if k.startswith(pre)}


def learner_case(i):
    z = npz("learner_traces")
    pre = f"l{i}_"
    return {k[len(pre):]: v for k, v in z.items() if k.startswith(pre)}


def noise_case(i):
    z = npz("noise_traces")
    pre = f"n{i}_"
    return {k[len(pre):]: v for k, v in z.items() if k.startswith(pre)}


def reward_plugin_inputs(i):
    """The arguments envs/manipulation_env.py:318-325 passed to reward_shaping.compute() at every
    step of golden env case i, rebuilt from the recorded trace: joint_positions = obs[:15] (the
    env's f32 array), contacts = obs[40:45], object_position = info["object_position"] (f64),
    finger_tips from the joints as _update_contacts builds them (ME:296-303).  Returns
    (jp [E][T][15] f32, tips [E][T][5][3] f64, op [E][T][3] f64, contacts [E][T][5] f32,
    length [E]); steps past an episode's length are padding."""
    z = env_case(i)
    obs = z["obs"]
    jp = obs[..., :15].astype(np.float32)
    s = jp.reshape(*jp.shape[:-1], 5, 3)
    s = ((s[..., 0] + s[..., 1]) + s[..., 2]).astype(np.float32)          # f32 sum in order
    tip = (s * np.float32(0.1)).astype(np.float64)                          # f32 * 0.1 (NEP 50) -> + zeros(3) f64
    tips = np.repeat(tip[..., None], 3, axis=-1)
    return jp, tips, z["op"].astype(np.float64), obs[..., 40:45].astype(np.float32), z["length"]
