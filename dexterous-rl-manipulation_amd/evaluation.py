"""Evaluation-side surfaces the hot path feeds (config C4/C5).

* ``HeldOutObjectSet`` / ``ObjectProperties`` / ``generate_training_objects``
  -- evaluation/heldout_objects.py:14-219.  Host-side object tables;
  ``native_table()`` turns them into device curriculum rows so env i of a
  vectorised evaluation gets object ``i % n`` (evaluator.py:215-223 order).
* ``NoisyObservationWrapper`` / ``NoisyDynamicsWrapper`` /
  ``CombinedNoiseWrapper`` -- evaluation/robustness_tests.py:15-211, for the
  single-env facade (one ``default_rng(seed)`` per wrapper, draws in the
  reference's order: dynamics noise before the step, observation noise
  after).  The vectorised trainer injects the same noise inside its fused
  rollout kernel instead.
* ``Evaluator`` / ``RobustnessTester`` (evaluator.py) and ``EvaluationMetrics`` /
  ``FailureType`` / ``format_metrics_report`` (metrics.py) are re-exported here
  under the reference's module path (evaluation/__init__.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from .experiments import CurriculumConfig


@dataclass
class ObjectProperties:
    size: float
    mass: float
    friction: float

    def _key(self):
        return (round(self.size, 4), round(self.mass, 4), round(self.friction, 4))

    def __hash__(self):
        return hash(self._key())

    def __eq__(self, other):
        return isinstance(other, ObjectProperties) and self._key() == other._key()


def _shifted_above(r):
    lo, hi = r
    return (hi + 0.01, hi + 0.01 + (hi - lo))


def _shifted_below(r):
    lo, hi = r
    return (max(0.0, lo - (hi - lo)), lo - 0.01)


class HeldOutObjectSet:
    """Evaluation objects disjoint from training (heldout_objects.py:39-189)."""

    def __init__(self, train_config: CurriculumConfig, eval_size_range: Optional[Tuple[float, float]] = None,
                 eval_mass_range: Optional[Tuple[float, float]] = None,
                 eval_friction_range: Optional[Tuple[float, float]] = None, num_heldout_objects: int = 20,
                 seed: int = 42):
        self.train_config = train_config
        self.num_heldout_objects = num_heldout_objects
        self.rng = np.random.default_rng(seed)
        # size/mass shift above the training range, friction below it (:70-95)
        if eval_size_range is None:
            eval_size_range = (_shifted_above(train_config.object_size_range) if train_config.object_size_range
                               else (0.06, 0.10))
        if eval_mass_range is None:
            eval_mass_range = (_shifted_above(train_config.object_mass_range) if train_config.object_mass_range
                               else (0.15, 0.25))
        if eval_friction_range is None:
            eval_friction_range = (_shifted_below(train_config.friction_range) if train_config.friction_range
                                   else (0.2, 0.4))
        self.eval_size_range = eval_size_range
        self.eval_mass_range = eval_mass_range
        self.eval_friction_range = eval_friction_range
        self.heldout_objects: List[ObjectProperties] = []
        self._generate_heldout_objects()

    def _generate_heldout_objects(self):
        u = self.rng.uniform
        for _ in range(self.num_heldout_objects):
            s = float(u(*self.eval_size_range))
            m = float(u(*self.eval_mass_range))
            f = float(u(*self.eval_friction_range))
            self.heldout_objects.append(ObjectProperties(size=s, mass=m, friction=f))

    def get_eval_config(self, object_idx: Optional[int] = None) -> CurriculumConfig:
        if object_idx is None:
            object_idx = self.rng.integers(0, len(self.heldout_objects))
        obj = self.heldout_objects[object_idx % len(self.heldout_objects)]
        t = self.train_config
        return CurriculumConfig(object_size=obj.size, object_mass=obj.mass, friction_coefficient=obj.friction,
                                spawn_distance=t.spawn_distance, spawn_distance_range=t.spawn_distance_range,
                                spawn_x_range=t.spawn_x_range, spawn_y_range=t.spawn_y_range,
                                spawn_z_range=t.spawn_z_range)

    def get_all_eval_configs(self) -> List[CurriculumConfig]:
        return [self.get_eval_config(i) for i in range(len(self.heldout_objects))]

    def native_table(self, num_envs: int):
        """(configs, env_index): env i evaluates object i % n."""
        cfgs = self.get_all_eval_configs()
        return cfgs, (np.arange(num_envs) % len(cfgs)).astype(np.int32)

    def verify_separation(self, train_objects: List[ObjectProperties]) -> bool:
        return len(set(train_objects) & set(self.heldout_objects)) == 0

    def get_statistics(self) -> Dict:
        a = np.array([[o.size, o.mass, o.friction] for o in self.heldout_objects])
        return {
            "num_objects": len(self.heldout_objects),
            "size_range": (float(a[:, 0].min()), float(a[:, 0].max())),
            "mass_range": (float(a[:, 1].min()), float(a[:, 1].max())),
            "friction_range": (float(a[:, 2].min()), float(a[:, 2].max())),
            "mean_size": float(np.mean(a[:, 0])),
            "mean_mass": float(np.mean(a[:, 1])),
            "mean_friction": float(np.mean(a[:, 2])),
        }


def generate_training_objects(config: CurriculumConfig, num_samples: int = 100,
                              seed: int = 42) -> List[ObjectProperties]:
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(num_samples):
        s = config.get_object_size(rng)
        m = config.get_object_mass(rng)
        f = config.get_friction_coefficient(rng)
        out.append(ObjectProperties(size=s, mass=m, friction=f))
    return out


# ------------------------------------------------------------------ noise wrappers
class _NoiseBase:
    def __init__(self, env, seed: Optional[int]):
        self.env = env
        self.rng = np.random.default_rng(seed)
        self.action_space = env.action_space
        self.observation_space = env.observation_space
        self.metadata = env.metadata

    def _obs_noise(self, obs: np.ndarray, std: float) -> np.ndarray:
        if std <= 0.0:
            return obs
        return obs + self.rng.normal(0, std, size=obs.shape).astype(obs.dtype)

    def _act_noise(self, action: np.ndarray, std: float) -> np.ndarray:
        if std <= 0.0:
            return action
        noisy = action + self.rng.normal(0, std, size=action.shape).astype(action.dtype)
        return np.clip(noisy, self.action_space.low, self.action_space.high)

    def close(self):
        self.env.close()


class NoisyObservationWrapper(_NoiseBase):
    """robustness_tests.py:15-77."""

    def __init__(self, env, observation_noise_std: float = 0.0, seed: Optional[int] = None):
        super().__init__(env, seed)
        self.observation_noise_std = observation_noise_std

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self._obs_noise(obs, self.observation_noise_std), info

    def step(self, action):
        obs, r, te, tr, info = self.env.step(action)
        return self._obs_noise(obs, self.observation_noise_std), r, te, tr, info


class NoisyDynamicsWrapper(_NoiseBase):
    """robustness_tests.py:80-137."""

    def __init__(self, env, dynamics_noise_std: float = 0.0, seed: Optional[int] = None):
        super().__init__(env, seed)
        self.dynamics_noise_std = dynamics_noise_std

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        return self.env.step(self._act_noise(action, self.dynamics_noise_std))


class CombinedNoiseWrapper(_NoiseBase):
    """robustness_tests.py:140-211."""

    def __init__(self, env, observation_noise_std: float = 0.0, dynamics_noise_std: float = 0.0,
                 seed: Optional[int] = None):
        super().__init__(env, seed)
        self.observation_noise_std = observation_noise_std
        self.dynamics_noise_std = dynamics_noise_std

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self._obs_noise(obs, self.observation_noise_std), info

    def step(self, action):
        obs, r, te, tr, info = self.env.step(self._act_noise(action, self.dynamics_noise_std))
        return self._obs_noise(obs, self.observation_noise_std), r, te, tr, info


_LAZY = {"Evaluator": "evaluator", "RobustnessTester": "evaluator", "EvaluationMetrics": "metrics",
         "FailureType": "metrics", "format_metrics_report": "metrics", "FailureMode": "failures",
         "FailureModeDefinition": "failures", "FAILURE_MODE_DEFINITIONS": "failures", "FailureClassifier": "failures",
         "FailureLogger": "failures", "EpisodeRecorder": "failures"}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module(f".{_LAZY[name]}", __package__), name)
    raise AttributeError(name)
