"""Policies -- policies/{simple_learner,random_policy,heuristic_policy}.py.

``SimpleLearner`` keeps the reference surface (``select_action(obs)``,
``update(reward)``, ``reset()``, ``mean_action``, ``best_reward``) and runs its
arithmetic in HIP kernels (``dxrl_learner_select`` / ``dxrl_learner_update``).
Its randomness is the reference's: the process-global legacy ``np.random``
stream (simple_learner.py:60,84), consumed on the host in the same order --
15 normals per action, 15 more only when the reward improves.

``VecSimpleLearner`` is the batched state (N independent learners) that the
fused rollout kernel (``dxrl_rollout_simple``) drives; see training.py.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from . import _native as N


class VecSimpleLearner:
    """Device state of N SimpleLearners: mean_action f32 [D][N], best f64 [N],
    open-episode return f64 [N], device-RNG counter u64 [N]."""

    def __init__(self, num_envs: int, action_dim: int = 15, learning_rate: float = 0.01,
                 exploration_noise: float = 0.3, action_clip_range: float = 0.5, seed: int = 0, device=None):
        self.device = N.require_gpu(device)
        self.num_envs = int(num_envs)
        self.action_dim = action_dim
        self.learning_rate = learning_rate
        self.exploration_noise = exploration_noise
        self.action_clip_range = action_clip_range
        self.seed = int(seed)
        lay = N.LearnerLayout()
        N.call("dxrl_learner_layout_for", self.num_envs, action_dim, C.byref(lay))
        self.layout = lay
        self._owner, self.state = N.aligned_empty(lay.total_bytes, self.device)
        self.init()

    def _stream(self):
        return N.stream_of(self.device)

    def init(self):
        N.call("dxrl_learner_init", self.device.index, self.num_envs, N.ptr(self.state), self._stream())

    def reset(self, mask: Optional[torch.Tensor] = None):
        N.call("dxrl_learner_reset", self.device.index, self.num_envs, N.ptr(self.state), N.ptr(mask),
               self._stream())

    def native_config(self):
        c = N.LearnerConfig()
        c.learning_rate = float(self.learning_rate)
        c.exploration_noise = float(self.exploration_noise)
        c.action_clip_range = float(self.action_clip_range)
        c.seed = self.seed & (2**64 - 1)
        return c

    def _view(self, off, count, dtype, shape):
        nbytes = count * torch.empty((), dtype=dtype).element_size()
        return self.state[off:off + nbytes].view(dtype).view(*shape)

    @property
    def mean_action(self) -> torch.Tensor:  # [D, N]
        return self._view(self.layout.mean, self.action_dim * self.num_envs, torch.float32,
                          (self.action_dim, self.num_envs))

    @property
    def best_reward(self) -> torch.Tensor:
        return self._view(self.layout.best, self.num_envs, torch.float64, (self.num_envs,))

    @property
    def episode_return(self) -> torch.Tensor:
        return self._view(self.layout.ep_return, self.num_envs, torch.float64, (self.num_envs,))

    def select(self, gauss: torch.Tensor, out: torch.Tensor):
        N.call("dxrl_learner_select", self.device.index, self.num_envs, N.ptr(self.state),
               float(self.exploration_noise), N.ptr(gauss), N.ptr(out), self._stream())
        return out

    def update(self, gauss: torch.Tensor, reward: torch.Tensor, mask: torch.Tensor):
        N.call("dxrl_learner_update", self.device.index, self.num_envs, N.ptr(self.state),
               float(self.learning_rate), float(self.action_clip_range), N.ptr(gauss), N.ptr(reward),
               N.ptr(mask), self._stream())


class SimpleLearner:
    """Drop-in for policies/simple_learner.py:13-99 (one learner)."""

    def __init__(self, action_space, learning_rate: float = 0.01, exploration_noise: float = 0.3,
                 action_clip_range: float = 0.5, device=None):
        self.action_space = action_space
        self.learning_rate = learning_rate
        self.exploration_noise = exploration_noise
        self.action_clip_range = action_clip_range
        d = int(action_space.shape[0])
        self._vec = VecSimpleLearner(1, d, learning_rate, exploration_noise, action_clip_range, device=device)
        self.best_reward = -np.inf
        dev = self._vec.device
        self._g = torch.empty(1, d, dtype=torch.float64, device=dev)
        self._a = torch.empty(1, d, dtype=torch.float32, device=dev)
        self._r = torch.empty(1, dtype=torch.float64, device=dev)
        self._one = torch.ones(1, dtype=torch.uint8, device=dev)

    @property
    def mean_action(self) -> np.ndarray:
        return self._vec.mean_action[:, 0].cpu().numpy()

    def select_action(self, observation: np.ndarray) -> np.ndarray:
        # np.random.normal(0, s, 15) == 0 + s * (15 legacy gauss draws)
        g = np.random.standard_normal(size=self._g.shape[1])
        self._g.copy_(torch.from_numpy(g).view(1, -1))
        self._vec.exploration_noise = self.exploration_noise
        self._vec.select(self._g, self._a)
        return self._a[0].cpu().numpy()

    def update(self, reward: float):
        if reward > self.best_reward:
            g = np.random.standard_normal(size=self._g.shape[1])
            self._g.copy_(torch.from_numpy(g).view(1, -1))
            self._r.fill_(float(reward))
            self._vec.learning_rate = self.learning_rate
            self._vec.action_clip_range = self.action_clip_range
            self._vec.update(self._g, self._r, self._one)
            self.best_reward = reward

    def reset(self):
        self.best_reward = -np.inf


class RandomPolicy:
    """policies/random_policy.py:13-44 -- samples the action space (whose RNG,
    like the reference's, is the Box's own; ``self.rng`` is kept but unused)."""

    def __init__(self, action_space, seed: Optional[int] = None):
        self.action_space = action_space
        self.rng = np.random.default_rng(seed)

    def select_action(self, observation: np.ndarray) -> np.ndarray:
        return self.action_space.sample()

    def reset(self):
        pass


class HeuristicPolicy:
    """policies/heuristic_policy.py:13-68 -- closing motion (-0.5) plus
    f32(U(-0.1, 0.1)) from the global np.random stream, clipped to the space."""

    def __init__(self, action_space, num_fingers: int = 5, joints_per_finger: int = 3):
        self.action_space = action_space
        self.num_fingers = num_fingers
        self.joints_per_finger = joints_per_finger
        self.num_joints = num_fingers * joints_per_finger

    def select_action(self, observation: np.ndarray) -> np.ndarray:
        action = np.full(self.num_joints, -0.5, dtype=np.float32)
        action += np.random.uniform(-0.1, 0.1, size=self.num_joints).astype(np.float32)
        return np.clip(action, self.action_space.low, self.action_space.high)

    def reset(self):
        pass
