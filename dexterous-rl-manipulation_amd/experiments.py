"""Configuration surfaces of the reference, kept loadable unchanged.

* ``CurriculumConfig``  -- experiments/config.py:17-217 (reset-time samplers,
  dict/JSON round trip, easy/medium/hard presets).  ``to_native()`` packs one
  row of the device curriculum table (include/dxrl.h ``dxrl_curriculum``).
* ``CurriculumScheduler`` / ``StepBasedScheduler`` --
  experiments/curriculum_scheduler.py:13-335.  Host-side and per-episode: the
  vectorised trainer feeds it finished episodes in (completion step, global
  env id) order and pushes the current config into the device table.
* ``ExperimentConfig`` tree + ``load_config`` / ``load_named_config`` --
  experiments/experiment_config.py:15-377, experiments/config_loader.py:13-66.
  Strict: unknown keys raise ``TypeError`` like ``cls(**d)`` does.

Build-owned knobs (num_envs, learner, bf16, world size ...) never go into
these dataclasses; they live in ``TrainerConfig`` (trainer.py).
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

Range = Optional[Tuple[float, float]]


# =============================================================== CurriculumConfig
@dataclass
class CurriculumConfig:
    object_size: float = 0.05
    object_size_range: Range = None
    object_mass: float = 0.1
    object_mass_range: Range = None
    friction_coefficient: float = 0.5
    friction_range: Range = None
    spawn_distance: float = 0.15
    spawn_distance_range: Range = None
    spawn_x_range: Tuple[float, float] = (-0.1, 0.1)
    spawn_y_range: Tuple[float, float] = (-0.1, 0.1)
    spawn_z_range: Tuple[float, float] = (0.05, 0.2)

    # -- samplers (config.py:44-113): one uniform draw each iff a range is set
    @staticmethod
    def _sample(rng, rng_range, const):
        if rng_range is None:
            return const
        return float(rng.uniform(rng_range[0], rng_range[1]))

    def get_object_size(self, rng) -> float:
        return self._sample(rng, self.object_size_range, self.object_size)

    def get_object_mass(self, rng) -> float:
        return self._sample(rng, self.object_mass_range, self.object_mass)

    def get_friction_coefficient(self, rng) -> float:
        return self._sample(rng, self.friction_range, self.friction_coefficient)

    def get_spawn_distance(self, rng) -> float:
        return self._sample(rng, self.spawn_distance_range, self.spawn_distance)

    def get_spawn_position(self, rng) -> Tuple[float, float, float]:
        return tuple(float(rng.uniform(r[0], r[1])) for r in (self.spawn_x_range, self.spawn_y_range,
                                                               self.spawn_z_range))

    # -- serialisation (config.py:115-172)
    _KEYS = ("object_size", "object_size_range", "object_mass", "object_mass_range", "friction_coefficient",
             "friction_range", "spawn_distance", "spawn_distance_range", "spawn_x_range", "spawn_y_range",
             "spawn_z_range")

    @classmethod
    def from_dict(cls, config_dict: dict) -> "CurriculumConfig":
        return cls(**config_dict)

    def to_dict(self) -> dict:
        return {k: getattr(self, k) for k in self._KEYS}

    @classmethod
    def from_json(cls, json_path: str) -> "CurriculumConfig":
        with open(json_path) as f:
            return cls.from_dict(json.load(f))

    def to_json(self, json_path: str):
        with open(json_path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    # -- presets (config.py:174-217) and the shipped JSON curricula
    @classmethod
    def easy(cls) -> "CurriculumConfig":
        return cls(object_size=0.08, object_mass=0.05, friction_coefficient=0.8, spawn_distance=0.10)

    @classmethod
    def medium(cls) -> "CurriculumConfig":
        return cls(object_size=0.05, object_mass=0.1, friction_coefficient=0.5, spawn_distance=0.15)

    @classmethod
    def hard(cls) -> "CurriculumConfig":
        return cls(object_size=0.03, object_mass=0.2, friction_coefficient=0.3, spawn_distance=0.20)

    @classmethod
    def variable(cls) -> "CurriculumConfig":
        """experiments/config_variable.json (domain-randomised ranges)."""
        return cls(object_size_range=(0.03, 0.07), object_mass_range=(0.05, 0.15), friction_range=(0.3, 0.7),
                   spawn_distance_range=(0.10, 0.20))

    @classmethod
    def named(cls, name: str) -> "CurriculumConfig":
        """config_{easy,medium,hard,variable}.json by name."""
        presets = {"easy": cls.easy, "medium": cls.medium, "hard": cls.hard, "variable": cls.variable,
                   "default": cls}
        if name not in presets:
            raise KeyError(f"unknown curriculum '{name}' (have {sorted(presets)})")
        return presets[name]()

    # -- device row
    def to_native(self):
        from ._native import Curriculum
        c = Curriculum()
        c.object_size = float(self.object_size)
        c.object_mass = float(self.object_mass)
        c.friction_coefficient = float(self.friction_coefficient)
        for name, flag, rng in (("size_range", "has_size_range", self.object_size_range),
                                ("mass_range", "has_mass_range", self.object_mass_range),
                                ("friction_range", "has_friction_range", self.friction_range)):
            if rng is not None:
                getattr(c, name)[0], getattr(c, name)[1] = float(rng[0]), float(rng[1])
                setattr(c, flag, 1)
        for name in ("spawn_x_range", "spawn_y_range", "spawn_z_range"):
            r = getattr(self, name)
            getattr(c, name)[0], getattr(c, name)[1] = float(r[0]), float(r[1])
        # NEP 50: a numpy.float64 friction turns `ov *= damping` into an f64 multiply
        # (a friction drawn from friction_range is a Python float)
        c.friction_is_f64_scalar = int(self.friction_range is None
                                       and isinstance(self.friction_coefficient, np.floating))
        return c


# ============================================================ curriculum schedulers
class CurriculumScheduler:
    """Success-rate driven difficulty progression (curriculum_scheduler.py:13-273).

    ``history``: "full" keeps every episode in ``episode_successes`` / ``episode_steps``
    as the reference does; "window" keeps only the last ``window_size`` of them (all the
    progression rule reads) plus counters, so a vectorised trainer feeding ~10^5-10^6
    episodes per iteration (``apply_device_summary``) does not grow host lists.  Totals,
    statistics and progression points are identical in both modes."""

    def __init__(self, initial_config: CurriculumConfig, target_config: CurriculumConfig,
                 success_rate_threshold: float = 0.7, min_episodes_before_progression: int = 50,
                 window_size: int = 20, progression_steps: int = 5, history: str = "full"):
        if history not in ("full", "window"):
            raise ValueError("history must be 'full' or 'window'")
        self.history = history
        self.initial_config = initial_config
        self.target_config = target_config
        self.success_rate_threshold = success_rate_threshold
        self.min_episodes_before_progression = min_episodes_before_progression
        self.window_size = window_size
        self.progression_steps = progression_steps
        self.reset()

    def _copy_config(self, config: CurriculumConfig) -> CurriculumConfig:
        return dataclasses.replace(config)

    def _interpolate_config(self, difficulty: float) -> CurriculumConfig:
        # np.clip returns numpy.float64, so the interpolated size/mass/friction
        # are numpy scalars -- kept on purpose (NEP 50 promotion in the step).
        d = np.clip(difficulty, 0.0, 1.0)
        a, b = self.initial_config, self.target_config

        def lerp(x, y):
            return x * (1 - d) + y * d

        size_range = None
        if a.object_size_range is not None and b.object_size_range is not None:
            size_range = (lerp(a.object_size_range[0], b.object_size_range[0]),
                          lerp(a.object_size_range[1], b.object_size_range[1]))
        return CurriculumConfig(
            object_size=lerp(a.object_size, b.object_size), object_size_range=size_range,
            object_mass=lerp(a.object_mass, b.object_mass), object_mass_range=a.object_mass_range,
            friction_coefficient=lerp(a.friction_coefficient, b.friction_coefficient),
            friction_range=a.friction_range,
            spawn_distance=lerp(a.spawn_distance, b.spawn_distance), spawn_distance_range=a.spawn_distance_range,
            spawn_x_range=a.spawn_x_range, spawn_y_range=a.spawn_y_range, spawn_z_range=a.spawn_z_range)

    def update(self, success: bool, episode_steps: int) -> bool:
        self.episode_successes.append(success)
        self.episode_steps.append(episode_steps)
        self.total_steps += episode_steps
        self.total_episodes += 1
        self._n_success += bool(success)
        progressed = self._progress() if self._should_progress() else False
        self._trim()
        return progressed

    def _trim(self):
        if self.history == "window" and len(self.episode_successes) > self.window_size:
            del self.episode_successes[:-self.window_size]
            del self.episode_steps[:-self.window_size]

    def _uses_success_window_rule(self) -> bool:
        """True when update / _should_progress / _progress are this class's (the rule the
        vectorised paths restate); subclasses such as StepBasedScheduler are fed per episode
        or through their own update_batch."""
        t = type(self)
        return (t.update is CurriculumScheduler.update and t._should_progress is CurriculumScheduler._should_progress
                and t._progress is CurriculumScheduler._progress and self.window_size > 0)

    def update_batch(self, successes, episode_steps) -> bool:
        """Exactly ``any([self.update(s, n) for s, n in zip(successes, episode_steps)])`` --
        same lists, totals, progression points and history entries -- without a Python call
        per episode (a 4096-env iteration finishes thousands of episodes).  The progression
        test depends only on the success window and the totals, so every candidate index is
        found with one cumulative sum; the difficulty only caps how many of them fire."""
        s = np.asarray(successes, dtype=bool).ravel()
        st = np.asarray(episode_steps, dtype=np.int64).ravel()
        if s.shape != st.shape:
            raise ValueError("successes and episode_steps must have the same length")
        n = s.size
        if n == 0:
            return False
        w = self.window_size
        if not self._uses_success_window_rule():  # other rules: per-episode calls
            return any([self.update(bool(a), int(b)) for a, b in zip(s, st)])
        base = self.total_episodes  # == len(episode_successes) with history="full"
        tail = np.asarray(self.episode_successes[-w:] if w > 0 else [], dtype=bool)
        hist = np.concatenate([tail, s])
        csum = np.concatenate([[0], np.cumsum(hist, dtype=np.int64)])
        k = np.arange(n)
        end = tail.size + k + 1                                     # hist prefix length after s[k]
        cnt = csum[end] - csum[np.maximum(end - w, 0)]
        ok = ((self.total_episodes + k + 1 >= self.min_episodes_before_progression) & (base + k + 1 >= w)
              & (cnt / w >= self.success_rate_threshold))
        steps_cum = np.cumsum(st)
        done, progressed = 0, False
        for j in np.nonzero(ok)[0]:
            if self.current_difficulty_level >= 1.0:
                break
            self.episode_successes.extend(s[done:j + 1].tolist())
            self.episode_steps.extend(st[done:j + 1].tolist())
            self.total_steps += int(steps_cum[j] - (steps_cum[done - 1] if done else 0))
            self.total_episodes += int(j + 1 - done)
            self._n_success += int(s[done:j + 1].sum())
            done = int(j + 1)
            progressed |= self._progress(rate=float(cnt[j]) / w)
        self.episode_successes.extend(s[done:].tolist())
        self.episode_steps.extend(st[done:].tolist())
        self.total_steps += int(steps_cum[-1] - (steps_cum[done - 1] if done else 0))
        self.total_episodes += int(n - done)
        self._n_success += int(s[done:].sum())
        self._trim()
        return progressed

    def remaining_progressions(self, cap: int) -> int:
        """How many more _progress calls can raise the level (at most cap + 1 is reported)."""
        lvl, n = self.current_difficulty_level, 0
        while lvl < 1.0 and n <= cap:
            new = min(lvl + 1.0 / self.progression_steps, 1.0)
            if new <= lvl:
                break
            lvl, n = new, n + 1
        return n

    def apply_device_summary(self, episodes: int, steps: int, successes: int, candidates, tail_codes,
                             episode_codes=None) -> bool:
        """Replay a batch summarised on the device (csrc/dxrl_sched.hip, dxrl_sched_scan):
        ``candidates`` = [(k, steps through k, window successes at k)] are the first episodes of
        the batch at which the progression test holds, in order; ``tail_codes`` the batch's
        last min(window, episodes) codes ((length << 1) | success) (history="window");
        ``episode_codes`` (history="full") every code of the batch.  Same totals, progression
        points and history entries as ``update_batch`` over the batch's (success, steps)."""
        if not self._uses_success_window_rule():
            raise ValueError("apply_device_summary restates CurriculumScheduler's success-window rule only")
        w = self.window_size
        e0, s0 = self.total_episodes, self.total_steps
        progressed = False
        for k, st_k, win in candidates:
            if self.current_difficulty_level >= 1.0:
                break
            self.total_episodes = e0 + int(k) + 1
            self.total_steps = s0 + int(st_k)
            progressed |= self._progress(rate=float(win) / w)
        self.total_episodes = e0 + int(episodes)
        self.total_steps = s0 + int(steps)
        self._n_success += int(successes)
        if episode_codes is not None:
            codes = np.asarray(episode_codes, dtype=np.int64)
            self.episode_successes.extend((codes & 1).astype(bool).tolist())
            self.episode_steps.extend((codes >> 1).tolist())
        else:
            if self.history == "full":
                raise ValueError("history='full' needs every episode code of the batch")
            tail = np.asarray(tail_codes, dtype=np.int64)[len(tail_codes) - min(w, int(episodes)):]
            self.episode_successes.extend((tail & 1).astype(bool).tolist())
            self.episode_steps.extend((tail >> 1).tolist())
        self._trim()
        return progressed

    def _window_rate(self):
        return np.mean(self.episode_successes[-self.window_size:])

    def _should_progress(self) -> bool:
        if self.total_episodes < self.min_episodes_before_progression:
            return False
        if self.current_difficulty_level >= 1.0:
            return False
        if self.total_episodes < self.window_size:  # == len(episode_successes) with history="full"
            return False
        return self._window_rate() >= self.success_rate_threshold

    def _progress(self, rate: Optional[float] = None) -> bool:
        """rate: the window success rate at this episode when the caller already has it
        (vectorised feeds); otherwise read from the list, as the reference does."""
        new = min(self.current_difficulty_level + 1.0 / self.progression_steps, 1.0)
        if new <= self.current_difficulty_level:
            return False
        self.current_difficulty_level = new
        self.current_config = self._interpolate_config(new)
        self.progression_history.append(
            self._history_entry(success_rate=float(self._window_rate()) if rate is None else float(rate)))
        return True

    def _history_entry(self, **extra):
        c = self.current_config
        entry = {"episode": self.total_episodes, "total_steps": self.total_steps}
        entry.update(extra)
        entry.update({"difficulty_level": float(self.current_difficulty_level),
                      "object_size": float(c.object_size), "object_mass": float(c.object_mass),
                      "friction_coefficient": float(c.friction_coefficient)})
        return entry

    def get_current_config(self) -> CurriculumConfig:
        return self.current_config

    def get_difficulty_level(self) -> float:
        return self.current_difficulty_level

    def get_statistics(self) -> Dict:
        n = self.total_episodes
        recent = self.episode_successes[-self.window_size:] if n >= self.window_size else self.episode_successes
        return {
            "total_episodes": self.total_episodes,
            "total_steps": self.total_steps,
            "current_difficulty_level": float(self.current_difficulty_level),
            "recent_success_rate": float(np.mean(recent)) if recent else 0.0,
            "overall_success_rate": self._n_success / n if n else 0.0,  # == np.mean(all successes)
            "num_progressions": len(self.progression_history),
            "progression_history": list(self.progression_history),
        }

    def reset(self):
        self.current_config = self._copy_config(self.initial_config)
        self.current_difficulty_level = 0.0
        self.episode_successes: List[bool] = []
        self.episode_steps: List[int] = []
        self.total_steps = 0
        self.total_episodes = 0
        self._n_success = 0
        self.progression_history: List[Dict] = []


class StepBasedScheduler(CurriculumScheduler):
    """Progress at total-step milestones (curriculum_scheduler.py:276-335)."""

    def __init__(self, initial_config, target_config, step_milestones: List[int], **kwargs):
        super().__init__(initial_config, target_config, **kwargs)
        self.step_milestones = sorted(step_milestones)
        self.current_milestone_idx = 0

    def _should_progress(self) -> bool:
        return (self.current_milestone_idx < len(self.step_milestones)
                and self.total_steps >= self.step_milestones[self.current_milestone_idx])

    def update_batch(self, successes, episode_steps) -> bool:
        """Exactly ``any([self.update(s, n) for ...])``: update() tests once per episode, so a
        milestone fires at the first episode whose running step total reaches it and at most
        one milestone fires per episode (the next one at a later episode at the earliest)."""
        t = type(self)
        if (t.update is not CurriculumScheduler.update or t._should_progress is not StepBasedScheduler._should_progress
                or t._progress is not StepBasedScheduler._progress):
            return super().update_batch(successes, episode_steps)
        s = np.asarray(successes, dtype=bool).ravel()
        st = np.asarray(episode_steps, dtype=np.int64).ravel()
        if s.shape != st.shape:
            raise ValueError("successes and episode_steps must have the same length")
        n = s.size
        if n == 0:
            return False
        cum = self.total_steps + np.cumsum(st)
        fire, j_prev = [], -1
        for m in self.step_milestones[self.current_milestone_idx:]:
            j = max(int(np.searchsorted(cum, m, side="left")), j_prev + 1)
            if j >= n:
                break
            fire.append(j)
            j_prev = j
        done, progressed = 0, False
        for j in fire:
            self.episode_successes.extend(s[done:j + 1].tolist())
            self.episode_steps.extend(st[done:j + 1].tolist())
            self.total_steps = int(cum[j])
            self.total_episodes += int(j + 1 - done)
            self._n_success += int(s[done:j + 1].sum())
            done = j + 1
            progressed |= self._progress()
        self.episode_successes.extend(s[done:].tolist())
        self.episode_steps.extend(st[done:].tolist())
        self.total_steps = int(cum[-1])
        self.total_episodes += int(n - done)
        self._n_success += int(s[done:].sum())
        self._trim()
        return progressed

    def _progress(self, rate: Optional[float] = None) -> bool:
        if self.current_milestone_idx >= len(self.step_milestones):
            return False
        self.current_milestone_idx += 1
        self.current_difficulty_level = min(self.current_milestone_idx / len(self.step_milestones), 1.0)
        self.current_config = self._interpolate_config(self.current_difficulty_level)
        self.progression_history.append(
            self._history_entry(milestone=self.step_milestones[self.current_milestone_idx - 1]))
        return True


# ============================================================ ExperimentConfig tree
class CurriculumLogger:
    """experiments/curriculum_logger.py:13-130: per-episode curriculum state and the
    scheduler's progression events, saved as JSON."""

    def __init__(self, log_dir: str = "logs"):
        from pathlib import Path
        self.log_dir = Path(log_dir)
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.episode_logs: List[Dict] = []
        self.progression_logs: List[Dict] = []

    def log_episode(self, episode: int, scheduler: CurriculumScheduler, success: bool, episode_steps: int):
        st = scheduler.get_statistics()
        c = scheduler.current_config
        self.episode_logs.append({
            "episode": episode, "total_steps": scheduler.total_steps,
            "difficulty_level": st["current_difficulty_level"], "success": success,
            "episode_steps": episode_steps, "recent_success_rate": st["recent_success_rate"],
            "object_size": c.object_size, "object_mass": c.object_mass,
            "friction_coefficient": c.friction_coefficient})

    def log_progression(self, scheduler: CurriculumScheduler, progression_occurred: bool):
        if progression_occurred and scheduler.progression_history:
            self.progression_logs.append(dict(scheduler.progression_history[-1]))

    def save(self, filename: str = "curriculum_progression.json"):
        path = self.log_dir / filename
        with open(path, "w") as f:
            json.dump({"episode_logs": self.episode_logs, "progression_logs": self.progression_logs}, f, indent=2)
        return path

    def print_progression_summary(self, scheduler: CurriculumScheduler):
        st = scheduler.get_statistics()
        bar = "=" * 60
        lines = ["\n" + bar, "Curriculum Progression Summary", bar,
                 f"Total episodes: {st['total_episodes']}", f"Total steps: {st['total_steps']}",
                 f"Current difficulty level: {st['current_difficulty_level']:.2f}",
                 f"Recent success rate: {st['recent_success_rate']:.3f}",
                 f"Overall success rate: {st['overall_success_rate']:.3f}",
                 f"Number of progressions: {st['num_progressions']}"]
        if self.progression_logs:
            lines += ["\nProgression History:", "-" * 60]
            for k, p in enumerate(self.progression_logs, 1):
                lines += [f"Progression {k}:", f"  Episode: {p.get('episode', 'N/A')}",
                          f"  Total steps: {p.get('total_steps', 'N/A')}",
                          f"  Difficulty level: {p.get('difficulty_level', 0):.2f}",
                          f"  Success rate: {p.get('success_rate', 0):.3f}",
                          f"  Object size: {p.get('object_size', 0):.4f} m",
                          f"  Object mass: {p.get('object_mass', 0):.4f} kg",
                          f"  Friction: {p.get('friction_coefficient', 0):.3f}", ""]
        lines.append(bar)
        print("\n".join(lines))


class _Section:
    """to_dict / strict from_dict shared by the experiment sections."""

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            out[f.name] = v.to_dict() if isinstance(v, _Section) else copy.copy(v)
        return out

    @classmethod
    def from_dict(cls, config_dict: Dict[str, Any]):
        d = dict(config_dict)
        for f in dataclasses.fields(cls):
            sub = _SECTION_TYPES.get(f.name)
            if sub is not None and f.name in d and isinstance(d[f.name], dict):
                d[f.name] = sub.from_dict(d[f.name])
        return cls(**d)  # unknown keys -> TypeError, like the reference


def _seeds(*s):
    return field(default_factory=lambda: list(s))


@dataclass
class TrainingConfig(_Section):
    num_episodes: int = 200
    max_episode_steps: int = 200
    learning_rate: float = 0.01
    seed: int = 42
    seeds: List[int] = _seeds(42, 123, 456, 789, 1000)
    reward_type: str = "dense"
    num_fingers: int = 5
    joints_per_finger: int = 3
    convergence_window_size: int = 20
    convergence_threshold: float = 0.5


@dataclass
class CurriculumSchedulerConfig(_Section):
    success_rate_threshold: float = 0.3
    window_size: int = 15
    min_episodes_before_progression: int = 20
    progression_steps: int = 5
    initial_difficulty: str = "easy"
    target_difficulty: str = "hard"


@dataclass
class EvaluationConfig(_Section):
    num_episodes_per_object: int = 5
    num_heldout_objects: int = 10
    max_episode_steps: int = 200
    seed: int = 42
    seeds: List[int] = _seeds(42, 123, 456, 789, 1000)
    reward_type: str = "dense"
    convergence_window_size: int = 20
    convergence_threshold: float = 0.5


@dataclass
class RobustnessConfig(_Section):
    observation_noise_levels: List[float] = _seeds(0.0, 0.01, 0.05, 0.1, 0.2)
    dynamics_noise_levels: List[float] = _seeds(0.0, 0.01, 0.05, 0.1, 0.2)
    num_episodes_per_noise: int = 10
    max_episode_steps: int = 200
    seed: int = 42


@dataclass
class SeedVarianceConfig(_Section):
    seeds: List[int] = _seeds(42, 123, 456, 789, 1000, 2024, 3000)
    num_episodes_per_object: int = 5
    max_episode_steps: int = 200
    max_cv_threshold: float = 0.2
    reward_type: str = "dense"

    def validate(self):
        if len(self.seeds) < 3:
            raise ValueError(f"Seed variance analysis requires at least 3 seeds, got {len(self.seeds)}")


@dataclass
class ComponentAblationConfig(_Section):
    num_episodes: int = 200
    max_episode_steps: int = 200
    seeds: List[int] = _seeds(42, 123, 456, 789, 1000)
    learning_rate: float = 0.01
    curriculum_scheduler: CurriculumSchedulerConfig = field(default_factory=CurriculumSchedulerConfig)


@dataclass
class ExperimentConfig(_Section):
    experiment_name: str = "default"
    description: str = ""
    training: TrainingConfig = field(default_factory=TrainingConfig)
    curriculum_scheduler: CurriculumSchedulerConfig = field(default_factory=CurriculumSchedulerConfig)
    evaluation: EvaluationConfig = field(default_factory=EvaluationConfig)
    robustness: RobustnessConfig = field(default_factory=RobustnessConfig)
    seed_variance: SeedVarianceConfig = field(default_factory=SeedVarianceConfig)
    component_ablation: ComponentAblationConfig = field(default_factory=ComponentAblationConfig)
    output_dir: str = "logs"

    def to_json(self, json_path: str):
        parent = os.path.dirname(json_path)
        if parent:
            os.makedirs(parent, exist_ok=True)
        with open(json_path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def from_json(cls, json_path: str) -> "ExperimentConfig":
        with open(json_path) as f:
            return cls.from_dict(json.load(f))

    @classmethod
    def default(cls) -> "ExperimentConfig":
        return cls(experiment_name="default", description="Default experiment configuration")

    @classmethod
    def quick_test(cls) -> "ExperimentConfig":
        return cls(experiment_name="quick_test", description="Quick test configuration with reduced parameters",
                   training=TrainingConfig(num_episodes=50, max_episode_steps=100, seeds=[42, 123]),
                   evaluation=EvaluationConfig(num_episodes_per_object=3, num_heldout_objects=5, seeds=[42, 123]),
                   seed_variance=SeedVarianceConfig(seeds=[42, 123, 456]),
                   component_ablation=ComponentAblationConfig(num_episodes=50, seeds=[42, 123]))


_SECTION_TYPES = {"training": TrainingConfig, "curriculum_scheduler": CurriculumSchedulerConfig,
                  "evaluation": EvaluationConfig, "robustness": RobustnessConfig,
                  "seed_variance": SeedVarianceConfig, "component_ablation": ComponentAblationConfig}


# The two ExperimentConfig JSONs the reference ships (experiments/config_default.json,
# experiments/config_quick_test.json), as section overrides of the defaults.
def _named_experiments() -> Dict[str, Dict[str, Any]]:
    sched_q = dict(window_size=10, min_episodes_before_progression=10, progression_steps=3)
    return {
        "default": dict(experiment_name="default",
                        description="Default experiment configuration for dexterous manipulation"),
        "quick_test": dict(
            experiment_name="quick_test",
            description="Quick test configuration with reduced parameters for fast testing",
            training=dict(num_episodes=50, max_episode_steps=100, seeds=[42, 123]),
            curriculum_scheduler=dict(sched_q),
            evaluation=dict(num_episodes_per_object=3, num_heldout_objects=5, max_episode_steps=100,
                            seeds=[42, 123], convergence_window_size=10),
            robustness=dict(observation_noise_levels=[0.0, 0.05, 0.1], dynamics_noise_levels=[0.0, 0.05, 0.1],
                            num_episodes_per_noise=5, max_episode_steps=100),
            seed_variance=dict(seeds=[42, 123, 456], num_episodes_per_object=3, max_episode_steps=100),
            component_ablation=dict(num_episodes=50, max_episode_steps=100, seeds=[42, 123],
                                    curriculum_scheduler=dict(sched_q)),
        ),
    }


CONFIG_DIR_ENV = "DXRL_CONFIG_DIR"


def load_config(config_path: Optional[str] = None) -> ExperimentConfig:
    """experiments/config_loader.py:13-30."""
    if config_path is None:
        return ExperimentConfig.default()
    if not os.path.exists(config_path):
        raise FileNotFoundError(f"Configuration file not found: {config_path}")
    return ExperimentConfig.from_json(config_path)


def get_config_path(config_name: str) -> str:
    """experiments/config_loader.py:33-52 -- looks in $DXRL_CONFIG_DIR."""
    d = os.environ.get(CONFIG_DIR_ENV, os.getcwd())
    p = os.path.join(d, f"config_{config_name}.json")
    if not os.path.exists(p):
        raise FileNotFoundError(f"Configuration '{config_name}' not found. Expected file: {p}")
    return p


def load_named_config(config_name: str) -> ExperimentConfig:
    """experiments/config_loader.py:55-66: the shipped names resolve without files."""
    try:
        return load_config(get_config_path(config_name))
    except FileNotFoundError:
        named = _named_experiments()
        if config_name not in named:
            raise
        base = ExperimentConfig().to_dict()
        for k, v in named[config_name].items():
            if isinstance(v, dict):
                sec = dict(base[k])
                for kk, vv in v.items():
                    sec[kk] = {**sec[kk], **vv} if isinstance(vv, dict) else vv
                base[k] = sec
            else:
                base[k] = v
        return ExperimentConfig.from_dict(base)
