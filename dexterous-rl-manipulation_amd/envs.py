"""Environments: the batched device env and the Gymnasium drop-in facade.

``VecEnv`` is N independent DexterousManipulationEnv replicas as one
struct-of-arrays slab in HBM, stepped by one HIP kernel launch
(``dxrl_env_step``) -- replaces envs/manipulation_env.py:184-252 for N envs.

``DexterousManipulationEnv`` keeps the reference's constructor, attributes,
``reset(seed, options) -> (obs, info)`` and
``step(action) -> (obs, reward, terminated, truncated, info)`` (numpy / Python
return types, envs/manipulation_env.py:24-349) on top of an N=1 ``VecEnv``.
The gymnasium RNG stays on the host exactly as in the reference (PCG64 seeded
through SeedSequence), so the host resolves reset draws in the reference's
order and the kernel consumes them -- bit-identical episodes for equal seeds.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .experiments import CurriculumConfig
from .rewards import resolve_plugin

NUM_FINGERS, JOINTS_PER_FINGER = 5, 3
ACTION_DIM = NUM_FINGERS * JOINTS_PER_FINGER
OBS_DIM = 2 * ACTION_DIM + 10 + NUM_FINGERS
RESET_SLOTS = ACTION_DIM + N.RESET_EXTRA

try:  # gymnasium is optional: the facade subclasses it when present
    import gymnasium as _gym
    from gymnasium import spaces as _spaces
    _EnvBase = _gym.Env
    Box = _spaces.Box
except ImportError:  # API-identical minimal stand-ins (gymnasium>=0.29 seeding semantics)
    _gym = None

    def _pcg(seed):
        return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))

    class _EnvBase:
        metadata: Dict[str, Any] = {}
        _np_random = None

        @property
        def np_random(self) -> np.random.Generator:
            if self._np_random is None:
                self._np_random = _pcg(None)
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = _pcg(seed)

        def close(self):
            pass

    class Box:
        """gymnasium.spaces.Box subset: bounds, dtype, shape, seed(), sample(), contains()."""

        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)
            self._np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = _pcg(None)
            return self._np_random

        def seed(self, seed=None):
            self._np_random = _pcg(seed)
            return [seed]

        def sample(self):
            return self.np_random.uniform(low=self.low, high=self.high, size=self.shape).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


def _curricula_table(configs: Sequence[Any]):
    arr = (N.Curriculum * len(configs))()
    for k, c in enumerate(configs):
        arr[k] = c.to_native() if hasattr(c, "to_native") else CurriculumConfig(**c.to_dict()).to_native()
    return arr


class VecEnv:
    """N env replicas on one GPU (one shard of a multi-GPU job).

    State: ``dxrl_env_layout`` SoA in a torch-owned HBM slab.  I/O tensors are
    preallocated; ``step`` returns views that the next call overwrites.
    """

    obs_dim = OBS_DIM
    action_dim = ACTION_DIM

    def __init__(self, num_envs: int, curriculum_config: Optional[CurriculumConfig] = None,
                 reward_type: str = "dense", reward_shaping=None, max_episode_steps: int = 200,
                 object_position: Optional[Sequence[float]] = None, seed: int = 0, device=None,
                 num_fingers: int = NUM_FINGERS, joints_per_finger: int = JOINTS_PER_FINGER,
                 global_env_offset: int = 0):
        self.device = N.require_gpu(device)
        kind, weights, self.reward_shaping = resolve_plugin(reward_type, reward_shaping)
        self.num_envs = int(num_envs)
        cfg = N.EnvConfig()
        cfg.num_envs = self.num_envs
        cfg.num_fingers, cfg.joints_per_finger = num_fingers, joints_per_finger
        cfg.max_episode_steps = int(max_episode_steps)
        cfg.reward_type = N.REWARD_DENSE if kind == "dense" else N.REWARD_SPARSE
        if object_position is not None:
            cfg.has_object_position = 1
            for k in range(3):
                cfg.object_position[k] = float(object_position[k])
        cfg.distance_weight, cfg.contact_weight, cfg.closure_weight, cfg.stability_weight = weights
        cfg.seed = int(seed) & (2**64 - 1)
        cfg.global_env_offset = int(global_env_offset)
        self._cfg = cfg
        self.reward_type = kind
        lay = N.EnvLayout()
        N.call("dxrl_env_layout_for", C.byref(cfg), C.byref(lay))
        self.layout = lay
        self._slab_owner, self.state = N.aligned_empty(lay.total_bytes, self.device)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            N.call("dxrl_env_create", C.byref(cfg), self.device.index, N.ptr(self.state), self._stream(), C.byref(h))
        self._h = h
        n, d = self.num_envs, ACTION_DIM
        dev = self.device
        self.obs = torch.empty(n, OBS_DIM, dtype=torch.float32, device=dev)
        self.reward = torch.empty(n, dtype=torch.float64, device=dev)
        self.terminated = torch.empty(n, dtype=torch.uint8, device=dev)
        self.truncated = torch.empty(n, dtype=torch.uint8, device=dev)
        self.components = torch.empty(n, 4, dtype=torch.float64, device=dev)
        self.curriculum_configs = [curriculum_config if curriculum_config is not None else CurriculumConfig()]
        self.set_curricula(self.curriculum_configs)

    # -- plumbing
    def _stream(self):
        return N.stream_of(self.device)

    def _view(self, off, count, dtype, shape):
        nbytes = count * torch.empty((), dtype=dtype).element_size()
        return self.state[off:off + nbytes].view(dtype).view(*shape)

    @property
    def handle(self):
        return self._h

    @property
    def max_episode_steps(self) -> int:
        return self._cfg.max_episode_steps

    @max_episode_steps.setter
    def max_episode_steps(self, v: int):
        self._cfg.max_episode_steps = int(v)
        N.call("dxrl_env_set_max_episode_steps", self._h, int(v))

    # -- curriculum (experiments/config.py rows; CurriculumScheduler pushes here)
    def set_curricula(self, configs: Sequence[Any], env_index: Optional[np.ndarray] = None):
        table = _curricula_table(configs)
        idx = None
        if env_index is not None:
            idx = np.ascontiguousarray(env_index, dtype=np.int32)
            if idx.shape != (self.num_envs,):
                raise ValueError(f"env_index must have shape ({self.num_envs},)")
        self.curriculum_configs = list(configs)
        with torch.cuda.device(self.device):
            N.call("dxrl_env_set_curricula", self._h, table, len(configs),
                   None if idx is None else idx.ctypes.data_as(C.c_void_p), self._stream())

    def set_curriculum(self, config):
        self.set_curricula([config])

    def set_curriculum_async(self, config):
        """``set_curriculum`` without a host sync (dxrl_env_set_curricula_async): the row is
        staged in a pinned buffer that the stream copies from; an event keeps the next call
        from overwriting it before the stream has passed the previous copy.  Every env uses
        row 0 afterwards, effective at its next reset."""
        if getattr(self, "_cur_stage", None) is None:
            self._cur_stage = torch.zeros(C.sizeof(N.Curriculum), dtype=torch.uint8).pin_memory()
            self._cur_event = torch.cuda.Event()
        self._cur_event.synchronize()  # the previous staged copy has been consumed
        row = config.to_native() if hasattr(config, "to_native") else CurriculumConfig(**config.to_dict()).to_native()
        C.memmove(self._cur_stage.data_ptr(), C.addressof(row), C.sizeof(row))
        self.curriculum_configs = [config]
        with torch.cuda.device(self.device):
            N.call("dxrl_env_set_curricula_async", self._h, self._cur_stage.data_ptr(), 1, None, self._stream())
            self._cur_event.record(torch.cuda.current_stream(self.device))

    # -- hot path
    def reset(self, mask: Optional[torch.Tensor] = None, draws: Optional[torch.Tensor] = None,
              write_obs: bool = True) -> torch.Tensor:
        """Reset the masked envs (all if mask is None).  draws: f64 [N, D+6] resolved
        reset draws (parity mode) or None (device Philox streams)."""
        if mask is not None:
            mask = self._check(mask, torch.uint8, (self.num_envs,), "mask")
        if draws is not None:
            draws = self._check(draws, torch.float64, (self.num_envs, RESET_SLOTS), "draws")
        N.call("dxrl_env_reset", self._h, N.ptr(mask), N.ptr(draws), N.ptr(self.obs) if write_obs else None,
               self._stream())
        return self.obs

    def step(self, actions: torch.Tensor, components: bool = False, write_obs: bool = True):
        actions = self._check(actions, torch.float32, (self.num_envs, ACTION_DIM), "actions")
        N.call("dxrl_env_step", self._h, N.ptr(actions), N.ptr(self.obs) if write_obs else None,
               N.ptr(self.reward), N.ptr(self.terminated), N.ptr(self.truncated),
               N.ptr(self.components) if components else None, self._stream())
        return self.obs, self.reward, self.terminated.view(torch.bool), self.truncated.view(torch.bool)

    def observe(self) -> torch.Tensor:
        N.call("dxrl_env_observe", self._h, N.ptr(self.obs), self._stream())
        return self.obs

    def _check(self, t, dtype, shape, name):
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor on {self.device}")
        if t.dtype != dtype:
            raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
        if tuple(t.shape) != shape:
            raise ValueError(f"{name} must have shape {shape}, got {tuple(t.shape)}")
        if t.device != self.device:
            raise ValueError(f"{name} must live on {self.device}, got {t.device}")
        if not t.is_contiguous() or t.data_ptr() % 16:
            t = t.contiguous().clone()
        return t

    # -- state views (read-only by convention)
    @property
    def joint_positions(self):
        return self._view(self.layout.jp, ACTION_DIM * self.num_envs, torch.float32, (ACTION_DIM, self.num_envs))

    @property
    def joint_velocities(self):
        return self._view(self.layout.jv, ACTION_DIM * self.num_envs, torch.float32, (ACTION_DIM, self.num_envs))

    @property
    def object_position(self):
        return self._view(self.layout.op, 3 * self.num_envs, torch.float64, (3, self.num_envs))

    @property
    def object_velocity(self):
        return self._view(self.layout.ov, 3 * self.num_envs, torch.float32, (3, self.num_envs))

    @property
    def flags(self):
        return self._view(self.layout.flags, self.num_envs, torch.int32, (self.num_envs,))

    @property
    def step_count(self):
        return self._view(self.layout.step_count, self.num_envs, torch.int32, (self.num_envs,))

    @property
    def object_size(self):
        return self._view(self.layout.size, self.num_envs, torch.float64, (self.num_envs,))

    @property
    def object_mass(self):
        return self._view(self.layout.mass, self.num_envs, torch.float64, (self.num_envs,))

    @property
    def friction_coefficient(self):
        return self._view(self.layout.friction, self.num_envs, torch.float64, (self.num_envs,))

    @property
    def curriculum_index(self):
        """Row of ``curriculum_configs`` each env resets from (i32 [N])."""
        return self._view(self.layout.cfg_index, self.num_envs, torch.int32, (self.num_envs,))

    @property
    def reset_counter(self):
        """Philox counter of each env's next device-RNG reset (u64 [N], as int64)."""
        return self._view(self.layout.reset_ctr, self.num_envs, torch.int64, (self.num_envs,))

    @property
    def contacts(self):
        bits = self.flags & 0xFF
        return torch.stack([(bits >> f) & 1 for f in range(NUM_FINGERS)], dim=1).to(torch.float32)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            torch.cuda.synchronize(self.device)
            N.lib().dxrl_env_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def resolve_reset_draws(rng: np.random.Generator, curriculum, first: bool, num_joints: int = ACTION_DIM):
    """Host mirror of the reference's reset-time RNG consumption
    (envs/manipulation_env.py:143-161): joints, then the curriculum's own
    get_object_size/mass/friction_coefficient, then -- only on the first reset
    of an instance -- get_spawn_position.  Returns (draw record, size, mass, friction)."""
    rec = np.full(num_joints + N.RESET_EXTRA, np.nan)
    rec[:num_joints] = rng.uniform(low=-0.1, high=0.1, size=(num_joints,))
    size = curriculum.get_object_size(rng)
    mass = curriculum.get_object_mass(rng)
    fric = curriculum.get_friction_coefficient(rng)
    rec[num_joints:num_joints + 3] = (size, mass, fric)
    if first:
        rec[num_joints + 3:] = curriculum.get_spawn_position(rng)
    return rec, size, mass, fric


class DexterousManipulationEnv(_EnvBase):
    """Drop-in for envs/manipulation_env.py:14-349 backed by the HIP kernels."""

    metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 30}
    _warned_f64 = False

    def __init__(self, num_fingers: int = 5, joints_per_finger: int = 3,
                 object_position: Optional[np.ndarray] = None, max_episode_steps: int = 200,
                 render_mode: Optional[str] = None, reward_type: str = "sparse", reward_shaping: Optional[Any] = None,
                 curriculum_config: Optional[Any] = None, device=None):
        super().__init__()
        self.num_fingers = num_fingers
        self.joints_per_finger = joints_per_finger
        self.num_joints = num_fingers * joints_per_finger
        self.render_mode = render_mode
        self.reward_type = reward_type
        self.curriculum_config = curriculum_config if curriculum_config is not None else CurriculumConfig()
        self._vec = VecEnv(1, reward_type=reward_type, reward_shaping=reward_shaping,
                           max_episode_steps=max_episode_steps, object_position=object_position, device=device,
                           num_fingers=num_fingers, joints_per_finger=joints_per_finger)
        self.reward_shaping = self._vec.reward_shaping
        self.action_space = Box(low=-1.0, high=1.0, shape=(self.num_joints,), dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(self._vec.obs_dim,), dtype=np.float32)
        self.workspace_bounds = np.array([[-0.2, 0.2], [-0.2, 0.2], [0.0, 0.3]])
        self.hand_base_position = np.array([0.0, 0.0, 0.0], dtype=np.float32)
        self._has_object = object_position is not None
        self.object_size = self.object_mass = self.friction_coefficient = None
        self.step_count = 0
        self._last_reward_components = None
        self._obs_dtype_f32 = True  # object_position dtype flips to f64 after the first step
        dev = self._vec.device
        self._draws = torch.empty(1, RESET_SLOTS, dtype=torch.float64, device=dev)
        self._act = torch.empty(1, ACTION_DIM, dtype=torch.float32, device=dev)
        # one packed D2H per step: obs f32[45] | reward f64 | comps f64[4] | op f64[3] | term, trunc
        self._io = torch.empty(512, dtype=torch.uint8, device=dev)
        self._pinned = torch.empty(512, dtype=torch.uint8).pin_memory()
        self._table_key = None

    @property
    def max_episode_steps(self) -> int:
        return self._vec.max_episode_steps

    @max_episode_steps.setter
    def max_episode_steps(self, v: int):
        self._vec.max_episode_steps = v

    def _sync_curriculum(self, fric):
        # every slot is resolved on the host, so the device row only needs
        # "take the slot" flags and the NEP-50 friction type of this episode
        f64 = isinstance(fric, np.floating)
        if self._table_key != f64:
            row = N.Curriculum()
            row.has_size_range = row.has_mass_range = row.has_friction_range = 1
            row.friction_is_f64_scalar = int(f64)
            table = (N.Curriculum * 1)(row)
            with torch.cuda.device(self._vec.device):
                N.call("dxrl_env_set_curricula", self._vec.handle, table, 1, None, self._vec._stream())
            self._table_key = f64

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None):
        super().reset(seed=seed)
        rec, size, mass, fric = resolve_reset_draws(self.np_random, self.curriculum_config,
                                                    first=not self._has_object, num_joints=self.num_joints)
        self._has_object = True
        self._sync_curriculum(fric)
        self.object_size, self.object_mass, self.friction_coefficient = size, mass, fric
        self._draws.copy_(torch.from_numpy(rec).view(1, -1), non_blocking=False)
        self._vec.reset(draws=self._draws)
        self.step_count = 0
        self.reward_shaping.reset()
        obs, op, _, _, _, _ = self._fetch(with_step=False)
        self._obs_dtype_f32 = True
        self._last_obs = obs
        return obs, self._info(op.astype(np.float32), obs)

    def step(self, action: np.ndarray):
        raw = np.asarray(action)
        if raw.dtype == np.float64 and not DexterousManipulationEnv._warned_f64:
            # NEP 50: the reference's `0.9 * jv + 0.1 * action` turns a float64 action into
            # float64 joint velocities (and positions) for the rest of the episode
            # (manipulation_env.py:203-205); the device state stays float32, so bit parity
            # holds for float32 actions (what Box.sample, SimpleLearner and the bundled
            # policies return).
            import warnings
            warnings.warn("DexterousManipulationEnv.step: float64 action cast to float32 (the reference would "
                          "carry float64 joint state; parity is defined for float32 actions)", RuntimeWarning,
                          stacklevel=2)
            DexterousManipulationEnv._warned_f64 = True
        a = raw.astype(np.float32, copy=False).reshape(1, self.num_joints)
        self._act.copy_(torch.from_numpy(a))
        self._vec.step(self._act, components=True)
        obs, op, reward, comps, term, trunc = self._fetch(with_step=True)
        self.step_count += 1
        self._last_reward_components = {"total": reward, "distance": comps[0], "contact": comps[1],
                                        "closure": comps[2], "stability": comps[3]}
        return obs, reward, term, trunc, self._info(op, obs)

    def _fetch(self, with_step: bool):
        v = self._vec
        io = self._io
        io[0:180].view(torch.float32).copy_(v.obs.view(-1))
        io[192:216].view(torch.float64).copy_(v.object_position.view(-1))
        if with_step:
            io[216:224].view(torch.float64).copy_(v.reward)
            io[224:256].view(torch.float64).copy_(v.components.view(-1))
            io[256:257].copy_(v.terminated)
            io[257:258].copy_(v.truncated)
        self._pinned.copy_(io)
        torch.cuda.current_stream(v.device).synchronize()
        h = self._pinned.numpy()
        obs = h[0:180].view(np.float32).copy()
        op = h[192:216].view(np.float64).copy()
        if not with_step:
            return obs, op, None, None, None, None
        reward = float(h[216:224].view(np.float64)[0])
        comps = [float(x) for x in h[224:256].view(np.float64)]
        return obs, op, reward, comps, bool(h[256]), bool(h[257])

    def _info(self, op, obs) -> Dict[str, Any]:
        info = {
            "step_count": self.step_count,
            "object_position": op,
            "num_contacts": int(np.sum(obs[2 * self.num_joints + 10:] > 0.5)),
            "curriculum": {
                "object_size": float(self.object_size),
                "object_mass": float(self.object_mass),
                "friction_coefficient": float(self.friction_coefficient),
            },
        }
        if self._last_reward_components is not None:
            info["reward_components"] = dict(self._last_reward_components)
        return info

    # -- reference attributes, read back from the device state
    def _col(self, t):
        return t[:, 0].cpu().numpy()

    @property
    def joint_positions(self):
        return self._col(self._vec.joint_positions)

    @property
    def joint_velocities(self):
        return self._col(self._vec.joint_velocities)

    @property
    def object_position(self):
        op = self._col(self._vec.object_position)
        return op.astype(np.float32) if self._obs_dtype_f32 and self.step_count == 0 else op

    @property
    def object_velocity(self):
        return self._col(self._vec.object_velocity)

    @property
    def object_orientation(self):
        return np.array([1.0, 0.0, 0.0, 0.0], dtype=np.float32)

    @property
    def contacts(self):
        return self._vec.contacts[0].cpu().numpy()

    @property
    def finger_tips(self):
        jp = self.joint_positions.reshape(self.num_fingers, self.joints_per_finger)
        s = np.array([np.sum(r) for r in jp], dtype=np.float32) * np.float32(0.1)
        return np.repeat(s.astype(np.float64)[:, None], 3, axis=1)

    def render(self):
        if self.render_mode == "rgb_array":
            return np.zeros((480, 640, 3), dtype=np.uint8)
        return None

    def close(self):
        self._vec.close()
