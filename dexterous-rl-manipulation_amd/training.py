"""Rollout drivers -- training/episode_utils.py:13-85, vectorised.

* ``run_episode`` / ``run_training_episode``: the reference loop, unchanged,
  for the Gymnasium facade (any env/policy pair with the reference's duck
  types).
* ``SimpleLearnerRollout``: N envs x N SimpleLearners advanced ``num_steps``
  steps per HIP launch (``dxrl_rollout_simple``), auto-resetting exactly like
  back-to-back ``run_episode`` calls, returning per-episode records in
  (completion step, global env id) order -- the order the host-side
  CurriculumScheduler is fed in.
* ``ReferenceStreams``: the reference's RNG streams per env (gymnasium PCG64
  for reset draws, legacy MT19937 ``np.random`` for the learner), turned into
  device tapes so a vectorised rollout reproduces N independent reference
  processes bit for bit.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .envs import ACTION_DIM, RESET_SLOTS, VecEnv, resolve_reset_draws
from .policies import VecSimpleLearner


# ------------------------------------------------------------------ reference loop
def run_episode(env, policy, max_steps: Optional[int] = None, reset_policy: bool = True) -> Tuple[bool, int, float]:
    """training/episode_utils.py:13-55 (success = info.get("success", False))."""
    obs, info = env.reset()
    if reset_policy and hasattr(policy, "reset"):
        policy.reset()
    max_steps = max_steps or env.max_episode_steps
    total_reward = 0.0
    success = False
    step = 0
    for step in range(max_steps):
        action = policy.select_action(obs)
        obs, reward, terminated, truncated, info = env.step(action)
        total_reward += reward
        if hasattr(policy, "update"):
            policy.update(reward)
        if terminated or truncated:
            success = info.get("success", False)
            break
    return success, step + 1, total_reward


def run_training_episode(env, policy, max_steps: Optional[int] = None) -> Dict[str, float]:
    """training/episode_utils.py:58-85."""
    success, steps, total_reward = run_episode(env, policy, max_steps=max_steps)
    return {"success": success, "steps": steps, "total_reward": total_reward,
            "mean_reward": total_reward / steps if steps > 0 else 0.0}


# ------------------------------------------------------------------ RNG mirrors
class ReferenceStreams:
    """Per-env reference RNG streams for parity-mode rollouts.

    env_seeds[i]     -> Generator(PCG64(SeedSequence(seed)))   (gymnasium np_random)
    learner_seeds[i] -> RandomState(seed) legacy gauss stream  (np.random.seed(seed))
    """

    def __init__(self, env: VecEnv, env_seeds: Sequence[int], learner_seeds: Sequence[int]):
        if len(env_seeds) != env.num_envs or len(learner_seeds) != env.num_envs:
            raise ValueError("one env seed and one learner seed per env")
        self.env = env
        self.rngs = [np.random.Generator(np.random.PCG64(np.random.SeedSequence(int(s)))) for s in env_seeds]
        self.legacy = [np.random.RandomState(int(s)) for s in learner_seeds]
        self.gbuf: List[np.ndarray] = [np.empty(0) for _ in env_seeds]
        # the first reset draws the spawn position only when the env was built without
        # object_position (manipulation_env.py:156-161)
        self.first = [not bool(env._cfg.has_object_position)] * env.num_envs

    def curriculum_of(self, i: int, env_index: Optional[np.ndarray]):
        row = 0 if env_index is None else int(env_index[i])
        return self.env.curriculum_configs[row]

    def initial_draws(self, env_index=None) -> torch.Tensor:
        recs = np.empty((self.env.num_envs, RESET_SLOTS))
        for i, rng in enumerate(self.rngs):
            recs[i], *_ = resolve_reset_draws(rng, self.curriculum_of(i, env_index), first=self.first[i])
            self.first[i] = False
        return torch.from_numpy(recs).to(self.env.device)

    def reset_tape(self, max_resets: int, env_index=None):
        """[N, max_resets*(D+6)] records + the generator states to rewind to."""
        n = self.env.num_envs
        tape = np.empty((n, max_resets * RESET_SLOTS))
        states = []
        for i, rng in enumerate(self.rngs):
            st = [rng.bit_generator.state]
            cur = self.curriculum_of(i, env_index)
            for k in range(max_resets):
                tape[i, k * RESET_SLOTS:(k + 1) * RESET_SLOTS], *_ = resolve_reset_draws(rng, cur, first=False)
                st.append(rng.bit_generator.state)
            states.append(st)
        return torch.from_numpy(tape).to(self.env.device), states

    def rewind(self, states, used: np.ndarray):
        for i, rng in enumerate(self.rngs):
            rng.bit_generator.state = states[i][int(used[i])]

    def gauss_tape(self, count: int) -> torch.Tensor:
        n = self.env.num_envs
        tape = np.empty((n, count))
        for i in range(n):
            need = count - len(self.gbuf[i])
            if need > 0:
                self.gbuf[i] = np.concatenate([self.gbuf[i], self.legacy[i].standard_normal(need)])
            tape[i] = self.gbuf[i][:count]
        return torch.from_numpy(tape).to(self.env.device)

    def consume_gauss(self, used: np.ndarray):
        for i in range(self.env.num_envs):
            self.gbuf[i] = self.gbuf[i][int(used[i]):]


# ------------------------------------------------------------------ fused rollout
@dataclass
class EpisodeRecords:
    """Finished episodes of one rollout call, in (end step, env id) order."""
    env_id: np.ndarray
    end_step: np.ndarray
    total_reward: np.ndarray
    steps: np.ndarray
    success: np.ndarray
    dropped: int = 0

    def __len__(self):
        return len(self.env_id)


class SimpleLearnerRollout:
    """run_episode x SimpleLearner for N envs, fused into one kernel per call."""

    def __init__(self, env: VecEnv, learner: VecSimpleLearner, max_steps: Optional[int] = None,
                 record_cap: int = 256, success_rule: str = "training",
                 streams: Optional[ReferenceStreams] = None):
        if learner.num_envs != env.num_envs or learner.device != env.device:
            raise ValueError("env and learner must have the same num_envs and device")
        if success_rule not in ("training", "terminated"):
            raise ValueError("success_rule must be 'training' (episode_utils.py:52) or 'terminated' "
                             "(evaluator.py:157)")
        self.env, self.learner = env, learner
        self.max_steps = max_steps or env.max_episode_steps
        self.success_rule = N.SUCCESS_TRAINING if success_rule == "training" else N.SUCCESS_TERMINATED
        self.streams = streams
        n, dev = env.num_envs, env.device
        self.record_cap = int(record_cap)
        self.ep_return = torch.empty(n, self.record_cap, dtype=torch.float64, device=dev)
        self.ep_length = torch.empty(n, self.record_cap, dtype=torch.int32, device=dev)
        self.ep_success = torch.empty(n, self.record_cap, dtype=torch.uint8, device=dev)
        self.ep_end = torch.empty(n, self.record_cap, dtype=torch.int32, device=dev)
        self.ep_count = torch.zeros(n, dtype=torch.int32, device=dev)
        self.gauss_used = torch.zeros(n, dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self._lcfg = learner.native_config()

    def start(self, env_index=None):
        """Episode 0 of every env: env.reset() + policy.reset() (episode_utils.py:33-36)."""
        draws = self.streams.initial_draws(env_index) if self.streams else None
        self.env.reset(draws=draws, write_obs=False)
        self.learner.reset()

    def run(self, num_steps: int, collect: bool = True, env_index=None,
            episode_budget: Optional[torch.Tensor] = None) -> Optional[EpisodeRecords]:
        """``num_steps`` steps of every env; ``episode_budget`` (i32 [N], device) stops an env
        once it has finished that many episodes in this call."""
        io = N.RolloutIO()
        io.episode_budget = N.ptr(episode_budget)
        io.record_cap = self.record_cap if collect else 0
        if collect:
            io.ep_return, io.ep_length = N.ptr(self.ep_return), N.ptr(self.ep_length)
            io.ep_success, io.ep_end_step = N.ptr(self.ep_success), N.ptr(self.ep_end)
            io.ep_count = N.ptr(self.ep_count)
        io.status = N.ptr(self.status)
        tapes = None
        if self.streams is not None:
            gcount = 2 * ACTION_DIM * num_steps
            gt = self.streams.gauss_tape(gcount)
            rt, states = self.streams.reset_tape(num_steps, env_index)
            tapes = (gt, rt, states)
            io.gauss, io.gauss_stride = N.ptr(gt), gcount
            io.reset_draws, io.reset_stride = N.ptr(rt), num_steps * RESET_SLOTS
            io.ep_count, io.gauss_used = N.ptr(self.ep_count), N.ptr(self.gauss_used)
        self.status.zero_()
        N.call("dxrl_rollout_simple", self.env.handle, N.ptr(self.learner.state), C.byref(self._lcfg),
               int(num_steps), int(self.max_steps), self.success_rule, C.byref(io), self.env._stream())
        if tapes is not None:
            counts = self.ep_count.cpu().numpy()
            self.streams.consume_gauss(self.gauss_used.cpu().numpy())
            self.streams.rewind(tapes[2], counts)
            if int(self.status.item()):
                raise N.NativeError("parity tape overrun in dxrl_rollout_simple")
        if not collect:
            return None
        return self.records()

    def records(self) -> EpisodeRecords:
        return gather_records(self.ep_count, self.record_cap, self.ep_return, self.ep_length, self.ep_success,
                              self.ep_end, self.env._cfg.global_env_offset)


def gather_records(count, cap, ret, length, success, end_step, gid0=0) -> EpisodeRecords:
    """Device [N][cap] episode records -> host EpisodeRecords in (end step, global env id)
    order, the order the host-side CurriculumScheduler is fed in."""
    counts = count.cpu().numpy().astype(np.int64)
    kept = np.minimum(counts, cap)
    n = counts.shape[0]
    m = np.arange(cap)[None, :] < kept[:, None]
    env_id = np.broadcast_to(np.arange(n)[:, None] + gid0, m.shape)[m]
    end = end_step.cpu().numpy()[m]
    order = np.lexsort((env_id, end))
    return EpisodeRecords(env_id=env_id[order], end_step=end[order], total_reward=ret.cpu().numpy()[m][order],
                          steps=length.cpu().numpy()[m][order],
                          success=success.cpu().numpy()[m][order].astype(bool), dropped=int((counts - kept).sum()))


# ------------------------------------------------------------------ JSON training log
class TrainingLogger:
    """training/logger.py:12-133: per-episode reward / steps / success series, a
    convergence episode (first reward above 0.5) and the JSON log format.
    ``log_records`` appends a device rollout's EpisodeRecords in one call
    (vectorised; the same series ``log_episode`` would build one by one)."""

    def __init__(self, log_dir: str = "logs", experiment_name: str = "experiment"):
        from pathlib import Path
        self.log_dir = Path(log_dir)
        self.experiment_name = experiment_name
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.convergence_threshold: float = 0.5
        self.reset()

    def reset(self):
        self.episode_rewards: List[float] = []
        self.episode_steps: List[int] = []
        self.success_rates: List[float] = []
        self.reward_components: List[Dict[str, float]] = []
        self.convergence_step: Optional[int] = None

    def log_episode(self, episode: int, reward: float, steps: int, success: bool,
                    reward_components: Optional[Dict[str, float]] = None):
        self.episode_rewards.append(reward)
        self.episode_steps.append(steps)
        self.success_rates.append(1.0 if success else 0.0)
        if reward_components:
            self.reward_components.append(dict(reward_components))
        if self.convergence_step is None and reward > self.convergence_threshold:
            self.convergence_step = episode

    def log_records(self, records: "EpisodeRecords", first_episode: Optional[int] = None):
        """Episodes of a rollout, in record order, numbered from ``first_episode``
        (default: continuing this log)."""
        base = len(self.episode_rewards) if first_episode is None else int(first_episode)
        rew = np.asarray(records.total_reward, dtype=np.float64)
        if self.convergence_step is None:
            hit = np.flatnonzero(rew > self.convergence_threshold)
            if len(hit):
                self.convergence_step = base + int(hit[0])
        self.episode_rewards += rew.tolist()
        self.episode_steps += np.asarray(records.steps).astype(np.int64).tolist()
        self.success_rates += np.where(np.asarray(records.success, dtype=bool), 1.0, 0.0).tolist()

    def get_statistics(self, window_size: int = 10) -> Dict[str, float]:
        if not self.episode_rewards:
            return {}
        r = self.episode_rewards
        s = self.success_rates
        rr, rs = r[-window_size:], s[-window_size:]
        return {"total_episodes": len(r), "mean_reward": float(np.mean(r)), "std_reward": float(np.std(r)),
                "recent_mean_reward": float(np.mean(rr)), "recent_std_reward": float(np.std(rr)),
                "overall_success_rate": float(np.mean(s)), "recent_success_rate": float(np.mean(rs)),
                "convergence_step": self.convergence_step,
                "mean_episode_steps": float(np.mean(self.episode_steps)) if self.episode_steps else 0.0}

    def save(self, filename: Optional[str] = None):
        import json
        path = self.log_dir / (filename or f"{self.experiment_name}_log.json")
        data = {"experiment_name": self.experiment_name, "statistics": self.get_statistics(),
                "episode_rewards": [float(x) for x in self.episode_rewards], "episode_steps": self.episode_steps,
                "success_rates": [float(x) for x in self.success_rates], "reward_components": self.reward_components}
        with open(path, "w") as f:
            json.dump(data, f, indent=2)
        return path
