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
