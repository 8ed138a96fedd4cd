"""Reward plugins -- rewards/reward_shaping.py:12-242.

The reference computes rewards in Python objects injected into the env
(envs/manipulation_env.py:64-73) and called once per step (:318-325).  Here both
built-in plugins are fused into the HIP step kernels; these classes carry the
plugin choice and the dense weights to the kernels, keep the reference's
constructor / attribute surface, and expose the reference's ``compute()`` for
callers outside ``env.step()`` -- evaluated on the GPU by ``dxrl_reward_compute``
(the step kernels' own ``dense_reward``), never on the CPU.

A subclass that overrides ``compute`` (or one of RewardShaping's ``_compute_*``
terms) cannot run inside the fused kernels: ``resolve_plugin`` rejects it with a
TypeError instead of silently computing the built-in reward.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import numpy as np

_KEYS = ("total", "distance", "contact", "closure", "stability")


def _device_compute(kind: int, weights, joint_positions, finger_tips, object_position, contacts, num_fingers,
                    joints_per_finger, state, device):
    """One batched dxrl_reward_compute launch.  Inputs: one item (the reference's shapes) or a
    leading batch axis; numpy arrays or torch tensors.  Returns (dict, batched, new state)."""
    import torch

    from . import _native as N
    dev = N.require_gpu(device)

    def dev_t(x, dt, tail):
        t = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
        t = t.to(device=dev, dtype=dt).contiguous()
        return t.reshape(-1, *tail) if t.dim() == len(tail) else t

    c = dev_t(contacts, torch.float32, (num_fingers,))
    batched = not (np.ndim(contacts) == 1 if not isinstance(contacts, torch.Tensor) else contacts.dim() == 1)
    B = c.shape[0]
    dense = kind == N.REWARD_DENSE
    jp = tips = op = prev = has = None
    w = None
    if dense:
        jp = dev_t(joint_positions, torch.float32, (num_fingers * joints_per_finger,))
        tips = dev_t(finger_tips, torch.float64, (num_fingers, 3))
        op = dev_t(object_position, torch.float64, (3,))
        if op.shape[0] == 1 and B > 1:
            op = op.expand(B, 3).contiguous()
        if not (jp.shape[0] == tips.shape[0] == op.shape[0] == B):
            raise ValueError("joint_positions, finger_tips, object_position and contacts disagree on the batch size")
        prev, has = state
        if prev is None:
            prev = torch.zeros(B, num_fingers, dtype=torch.float32, device=dev)
            has = torch.zeros(B, dtype=torch.uint8, device=dev)
        elif prev.shape[0] != B:
            raise ValueError(f"batch size changed from {prev.shape[0]} to {B} while prev_contacts is set: call "
                             "reset() first (the stability term compares each row with its own previous contacts)")
        else:
            # the kernel updates the previous contacts in place; the tensor handed out as
            # prev_contacts after the last call (or assigned by the caller) must stay as it was,
            # as the reference's contacts.copy() leaves it (reward_shaping.py:174,185)
            prev, has = prev.clone(), has.clone()
        w = (C.c_double * 4)(*weights)
    out = torch.empty(B, 5, dtype=torch.float64, device=dev)
    N.call("dxrl_reward_compute", dev.index, kind, w, B, num_fingers, joints_per_finger, N.ptr(jp), N.ptr(tips),
           N.ptr(op), N.ptr(c), N.ptr(prev), N.ptr(has), N.ptr(out), N.stream_of(dev))
    if batched:
        res = {k: out[:, j] for j, k in enumerate(_KEYS)}
    else:
        o = out[0].tolist()
        res = {k: o[j] for j, k in enumerate(_KEYS)}
    return res, batched, (prev, has)


class RewardShaping:
    """Dense shaping: w_d*exp(-5*min d) + w_c*contacts/F + w_cl*closure + w_s*stability
    (reward_shaping.py:50-187).  Evaluated inside the step kernel; ``compute`` runs the same
    device function on caller-given inputs."""

    native_kind = "dense"

    def __init__(self, distance_weight: float = 1.0, contact_weight: float = 0.5, closure_weight: float = 0.3,
                 stability_weight: float = 0.2, device=None):
        self.distance_weight = distance_weight
        self.contact_weight = contact_weight
        self.closure_weight = closure_weight
        self.stability_weight = stability_weight
        self.device = device  # where compute() runs (None: the current GPU)
        # reward_shaping.py:41-43.  Inside an env the per-env previous-contact state lives in the
        # device flag word; compute() keeps its own (device f32 [B][5] + has-prev bytes).
        self.prev_contacts: Optional[object] = None
        self.prev_distances: Optional[object] = None
        self._state, self._prev_obj = (None, None), None

    def reset(self):
        """reward_shaping.py:45-48."""
        self.prev_contacts = None
        self.prev_distances = None
        self._state, self._prev_obj = (None, None), None

    @property
    def weights(self):
        return (float(self.distance_weight), float(self.contact_weight), float(self.closure_weight),
                float(self.stability_weight))

    def compute(self, joint_positions, finger_tips, object_position, contacts, num_fingers: int = 5,
                joints_per_finger: int = 3) -> Dict[str, float]:
        """reward_shaping.py:50-99 on the GPU.  One item (joint_positions (15,), finger_tips
        (5, 3), object_position (3,), contacts (5,)) returns the reference's dict of floats;
        a leading batch axis returns f64 device tensors [B] per key and keeps one
        prev-contacts state per row.  joint_positions / contacts are taken as f32 (the env's
        arrays, manipulation_env.py:143-145, :310), finger_tips / object_position as f64."""
        from . import _native as N
        if self.prev_contacts is None:
            self._state = (None, None)
        elif self.prev_contacts is not self._prev_obj:  # prev_contacts assigned from outside
            self._state = self._state_from_host(self.prev_contacts, num_fingers)
        res, batched, st = _device_compute(N.REWARD_DENSE, self.weights, joint_positions, finger_tips,
                                           object_position, contacts, num_fingers, joints_per_finger, self._state,
                                           self.device)
        self._state = st
        # reward_shaping.py:174,185: prev_contacts = contacts.copy()
        self.prev_contacts = self._prev_obj = st[0][0].cpu().numpy() if not batched else st[0]
        return res

    def _state_from_host(self, prev, F):
        import torch

        from . import _native as N
        dev = N.require_gpu(self.device)
        p = torch.as_tensor(np.asarray(prev) if not isinstance(prev, torch.Tensor) else prev)
        p = p.to(device=dev, dtype=torch.float32).reshape(-1, F).clone()  # never the caller's own tensor
        return p, torch.ones(p.shape[0], dtype=torch.uint8, device=dev)


class SparseReward:
    """+1 when >= 3 fingers touch, else -0.01 (reward_shaping.py:190-242)."""

    native_kind = "sparse"
    weights = (1.0, 0.5, 0.3, 0.2)  # unused by the sparse kernel path

    def __init__(self, device=None):
        self.device = device

    def reset(self):
        pass

    def compute(self, joint_positions, finger_tips, object_position, contacts, num_fingers: int = 5,
                joints_per_finger: int = 3) -> Dict[str, float]:
        """reward_shaping.py:205-242 on the GPU (only `contacts` is read)."""
        from . import _native as N
        res, _, _ = _device_compute(N.REWARD_SPARSE, None, None, None, None, contacts, num_fingers,
                                    joints_per_finger, (None, None), self.device)
        return res


# the methods whose behaviour the fused kernels implement: overriding any of them changes the
# reward the reference would compute, which the kernels cannot follow
_FUSED_METHODS = {
    "dense": (RewardShaping, ("compute", "_compute_distance_reward", "_compute_contact_reward",
                              "_compute_closure_reward", "_compute_stability_reward")),
    "sparse": (SparseReward, ("compute",)),
}


def resolve_plugin(reward_type: str, reward_shaping):
    """envs/manipulation_env.py:64-73 plugin choice -> (kind, weights, plugin)."""
    plugin = reward_shaping
    if plugin is None:
        plugin = RewardShaping() if reward_type == "dense" else SparseReward()
    kind = getattr(plugin, "native_kind", None)
    if kind not in ("dense", "sparse"):
        raise TypeError("reward_shaping must be a RewardShaping or SparseReward instance: the reward is fused into "
                        "the HIP step kernel (custom Python reward plugins are not supported)")
    base, names = _FUSED_METHODS[kind]
    if not isinstance(plugin, base):
        raise TypeError(f"reward_shaping declares native_kind={kind!r} but is not a {base.__name__}")
    for name in names:
        if getattr(type(plugin), name, None) is not getattr(base, name, None):
            raise TypeError(f"{type(plugin).__name__} overrides {name}(): the {kind} reward is fused into the HIP "
                            "step kernels, which cannot run a Python override (custom reward plugins are not "
                            "supported; use RewardShaping / SparseReward or their weights)")
    return kind, plugin.weights, plugin
