"""Reward plugins -- rewards/reward_shaping.py:12-242.

The reference computes rewards in Python objects injected into the env
(envs/manipulation_env.py:64-73).  Here both built-in plugins are fused into
the HIP step kernel; these classes carry the plugin choice and the dense
weights to the kernel and keep the reference's constructor/attribute surface.
"""
from __future__ import annotations

from typing import Optional


class RewardShaping:
    """Dense shaping: w_d*exp(-5*min d) + w_c*contacts/F + w_cl*closure + w_s*stability
    (reward_shaping.py:50-187).  Evaluated inside the step kernel."""

    native_kind = "dense"

    def __init__(self, distance_weight: float = 1.0, contact_weight: float = 0.5, closure_weight: float = 0.3,
                 stability_weight: float = 0.2):
        self.distance_weight = distance_weight
        self.contact_weight = contact_weight
        self.closure_weight = closure_weight
        self.stability_weight = stability_weight
        # the per-env previous-contact state lives in the device flag word
        self.prev_contacts: Optional[object] = None
        self.prev_distances: Optional[object] = None

    def reset(self):
        self.prev_contacts = None
        self.prev_distances = None

    @property
    def weights(self):
        return (float(self.distance_weight), float(self.contact_weight), float(self.closure_weight),
                float(self.stability_weight))


class SparseReward:
    """+1 when >= 3 fingers touch, else -0.01 (reward_shaping.py:190-242)."""

    native_kind = "sparse"
    weights = (1.0, 0.5, 0.3, 0.2)  # unused by the sparse kernel path

    def reset(self):
        pass


def resolve_plugin(reward_type: str, reward_shaping):
    """envs/manipulation_env.py:64-73 plugin choice -> (kind, weights, plugin)."""
    plugin = reward_shaping
    if plugin is None:
        plugin = RewardShaping() if reward_type == "dense" else SparseReward()
    kind = getattr(plugin, "native_kind", None)
    if kind not in ("dense", "sparse"):
        raise TypeError("reward_shaping must be a RewardShaping or SparseReward instance: the reward is fused into "
                        "the HIP step kernel (custom Python reward plugins are not supported)")
    return kind, plugin.weights, plugin
