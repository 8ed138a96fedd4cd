"""Failure taxonomy and failure-episode logs.

* ``FailureMode`` / ``FailureModeDefinition`` / ``FAILURE_MODE_DEFINITIONS`` /
  ``FailureClassifier`` -- evaluation/failure_taxonomy.py:14-318.  The rule
  order and thresholds are the reference's; the numeric parts of the
  definitions (``detection_criteria``) are the values the rules read.
* ``FailureLogger`` / ``EpisodeRecorder`` -- evaluation/failure_logger.py:14-297,
  the JSON trajectory log format.  The device evaluator (evaluator.py) fills
  them from its episode buffers: per-step contact counts and, for logged
  episodes, the observation / action trajectories ``k_eval`` records.

The classifier's statistics (variance, trend) go through the same NumPy calls on
the same integer lists as the reference, so classifications and confidences are
the reference's bit for bit (tests/golden/eval_golden.json "taxonomy").
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from datetime import datetime
from enum import Enum
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import numpy as np


class FailureMode(Enum):
    """failure_taxonomy.py:14-27."""
    SLIPPAGE = "slippage"
    UNSTABLE_GRASP = "unstable_grasp"
    MISALIGNMENT = "misalignment"
    TIMEOUT = "timeout"
    OBJECT_DROPPED = "object_dropped"
    INSUFFICIENT_CONTACTS = "insufficient_contacts"


@dataclass
class FailureModeDefinition:
    """failure_taxonomy.py:30-40."""
    mode: FailureMode
    name: str
    description: str
    key_indicators: List[str]
    detection_criteria: Dict


def _definition(mode, name, description, indicators, criteria):
    return mode, FailureModeDefinition(mode, name, description, indicators, criteria)


# failure_taxonomy.py:43-135 -- names and detection criteria as the classifier reads them
FAILURE_MODE_DEFINITIONS: Dict[FailureMode, FailureModeDefinition] = dict([
    _definition(FailureMode.SLIPPAGE, "Slippage",
                "The object slides out of the grasp after contact was made.",
                ["contact count falls over the episode", "contacts lost after being made"],
                {"contact_trend_threshold": -1.0, "min_contacts_for_slippage": 1, "contact_loss_threshold": 0.5}),
    _definition(FailureMode.UNSTABLE_GRASP, "Unstable Grasp",
                "Contacts form but the contact count fluctuates strongly.",
                ["high variance of the contact count", "frequent contact changes"],
                {"contact_variance_threshold": 2.0, "min_episode_length": 10, "contact_fluctuation_threshold": 3}),
    _definition(FailureMode.MISALIGNMENT, "Misalignment",
                "Some fingers touch the object, too few for a grasp.",
                ["1-2 stable contacts", "grasp never completes"],
                {"min_contacts": 1, "max_contacts": 2, "contact_stability": True}),
    _definition(FailureMode.TIMEOUT, "Timeout",
                "The episode hit its step limit without a grasp.",
                ["episode length equals the limit", "no grasp"],
                {"episode_length_equals_max": True, "success": False}),
    _definition(FailureMode.OBJECT_DROPPED, "Object Dropped",
                "All contacts were lost after some had been made.",
                ["zero final contacts", "contacts existed earlier"],
                {"final_contacts": 0, "had_contacts_before": True}),
    _definition(FailureMode.INSUFFICIENT_CONTACTS, "Insufficient Contacts",
                "The hand never reached enough contacts to grasp.",
                ["contact count always below the threshold"],
                {"max_contacts_below_threshold": True, "never_reached_threshold": True}),
])


def _counts_of(history) -> List[int]:
    return [len([c for c in row if c > 0.5]) for row in history]


class FailureClassifier:
    """failure_taxonomy.py:138-318: heuristic mapping of a failed episode to a mode."""

    def __init__(self, success_threshold: int = 3):
        self.success_threshold = success_threshold
        self.definitions = FAILURE_MODE_DEFINITIONS

    def classify(self, episode_data: Dict, max_steps: int = 200) -> Tuple[Optional[FailureMode], Dict]:
        if episode_data.get("success", False):
            return None, {}
        steps = episode_data.get("episode_steps", 0)
        nc = episode_data.get("num_contacts", 0)
        final = episode_data.get("final_contacts", nc)
        counts = _counts_of(episode_data.get("contact_history", []))
        peak = max(counts) if counts else nc
        var = np.var(counts) if len(counts) > 1 else 0.0
        crit = {m: d.detection_criteria for m, d in self.definitions.items()}
        if steps >= max_steps:                                             # :191-194
            return FailureMode.TIMEOUT, {"timeout": 1.0}
        if final == 0 and peak > 0:                                        # :196-199
            return FailureMode.OBJECT_DROPPED, {"object_dropped": 1.0}
        if len(counts) > 5:                                                # :202-221
            if len(counts) > 10:
                trend = np.mean(counts[-5:]) - np.mean(counts[:5])
                c = crit[FailureMode.SLIPPAGE]
                if trend < c["contact_trend_threshold"] and peak >= c["min_contacts_for_slippage"]:
                    return FailureMode.SLIPPAGE, {"slippage": min(1.0, abs(trend) / 2.0)}
            if var > crit[FailureMode.UNSTABLE_GRASP]["contact_variance_threshold"]:
                return FailureMode.UNSTABLE_GRASP, {"unstable_grasp": min(1.0, var / 5.0)}
        c = crit[FailureMode.MISALIGNMENT]                                 # :223-229
        if c["min_contacts"] <= nc <= c["max_contacts"] and var < 1.0:
            return FailureMode.MISALIGNMENT, {"misalignment": 0.8}
        if peak < self.success_threshold:                                  # :231-234
            return FailureMode.INSUFFICIENT_CONTACTS, {"insufficient_contacts": 1.0}
        return FailureMode.INSUFFICIENT_CONTACTS, {"insufficient_contacts": 0.5}

    def get_failure_mode_info(self, mode: FailureMode) -> FailureModeDefinition:
        return self.definitions[mode]

    def classify_batch(self, episodes: List[Dict], max_steps: int = 200) -> Dict:
        """:253-281 (annotates each episode dict in place)."""
        out: Dict[Any, List[Dict]] = {m: [] for m in FailureMode}
        out[None] = []
        for ep in episodes:
            mode, conf = self.classify(ep, max_steps)
            ep["failure_mode"] = mode.value if mode else None
            ep["failure_confidence"] = conf
            out[mode].append(ep)
        return out

    def get_failure_statistics(self, episodes: List[Dict], max_steps: int = 200) -> Dict:
        """:283-318."""
        by_mode = self.classify_batch(episodes, max_steps)
        total = len(episodes)
        ok = len(by_mode[None])
        counts = {m.value: len(v) for m, v in by_mode.items() if m is not None}
        return {"total_episodes": total, "successful_episodes": ok, "failed_episodes": total - ok,
                "success_rate": ok / total if total > 0 else 0.0, "failure_counts": counts,
                "failure_frequencies": {k: v / total for k, v in counts.items()},
                "classified_episodes": by_mode}


def _plain(obj: Any) -> Any:
    """JSON-ready copy: numpy scalars / arrays to Python numbers / lists."""
    if isinstance(obj, (bool, np.bool_)):
        return bool(obj)
    if isinstance(obj, np.integer):
        return int(obj)
    if isinstance(obj, np.floating):
        return float(obj)
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    return obj


class FailureLogger:
    """failure_logger.py:14-239: failure episodes with trajectories, saved as JSON."""

    def __init__(self, log_dir: str = "logs/failures", save_full_trajectories: bool = True,
                 success_threshold: int = 3):
        self.log_dir = Path(log_dir)
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.save_full_trajectories = save_full_trajectories
        self.classifier = FailureClassifier(success_threshold=success_threshold)
        self.logged_episodes: List[Dict] = []
        self.episode_counter = 0

    def log_episode(self, episode_data: Dict, states=None, actions=None, contacts=None,
                    metadata: Optional[Dict] = None, max_steps: int = 200) -> Dict:
        mode, conf = self.classifier.classify(episode_data, max_steps=max_steps)
        history = episode_data.get("contact_history", []) if contacts is None else contacts
        g = episode_data.get
        entry = {
            "episode_id": self.episode_counter,
            "timestamp": datetime.now().isoformat(),
            "success": g("success", False),
            "failure_mode": mode.value if mode else None,
            "failure_confidence": conf,
            "episode_steps": g("episode_steps", 0),
            "episode_reward": g("episode_reward", 0.0),
            "num_contacts": g("num_contacts", 0),
            "final_contacts": g("final_contacts", g("num_contacts", 0)),
            "contact_history": [[float(c) for c in row] for row in history] if history else [],
            "object_properties": {"size": g("object_size", 0.0), "mass": g("object_mass", 0.0),
                                  "friction_coefficient": g("friction_coefficient", 0.0)},
            "metadata": metadata or {},
        }
        if self.save_full_trajectories:
            if states is not None:
                entry["states"] = [s.tolist() if isinstance(s, np.ndarray) else s for s in states]
            if actions is not None:
                entry["actions"] = [a.tolist() if isinstance(a, np.ndarray) else a for a in actions]
        self.logged_episodes.append(entry)
        self.episode_counter += 1
        return entry

    def _mode_counts(self) -> Dict[str, int]:
        counts: Dict[str, int] = {}
        for ep in self.logged_episodes:
            m = ep.get("failure_mode")
            if m:
                counts[m] = counts.get(m, 0) + 1
        return counts

    def save(self, filename: Optional[str] = None) -> Path:
        if filename is None:
            filename = f"failures_{datetime.now().strftime('%Y%m%d_%H%M%S')}.json"
        path = self.log_dir / filename
        data = {"metadata": {"total_episodes": len(self.logged_episodes), "failure_modes": self._mode_counts(),
                             "logged_at": datetime.now().isoformat()},
                "episodes": _plain(self.logged_episodes)}
        with open(path, "w") as f:
            json.dump(data, f, indent=2)
        return path

    def load(self, filepath: str) -> Dict:
        with open(filepath) as f:
            data = json.load(f)
        self.logged_episodes = data.get("episodes", [])
        self.episode_counter = max((ep["episode_id"] for ep in self.logged_episodes), default=-1) + 1
        return data

    def get_statistics(self) -> Dict:
        if not self.logged_episodes:
            return {}
        lengths = [ep["episode_steps"] for ep in self.logged_episodes]
        rewards = [ep["episode_reward"] for ep in self.logged_episodes]
        return {"total_episodes": len(self.logged_episodes), "failure_mode_counts": self._mode_counts(),
                "mean_episode_length": float(np.mean(lengths)) if lengths else 0.0,
                "mean_reward": float(np.mean(rewards)) if rewards else 0.0}

    def reset(self):
        self.logged_episodes = []
        self.episode_counter = 0


class EpisodeRecorder:
    """failure_logger.py:242-297: per-step trajectory buffer of one episode."""

    def __init__(self, record_states: bool = True, record_actions: bool = True):
        self.record_states = record_states
        self.record_actions = record_actions
        self.reset()

    def record_step(self, state=None, action=None, contacts=None):
        if self.record_states and state is not None:
            self.states.append(state.copy())
        if self.record_actions and action is not None:
            self.actions.append(action.copy())
        if contacts is not None:
            self.contacts.append([float(c) for c in contacts])

    def set_metadata(self, **kwargs):
        self.metadata.update(kwargs)

    def get_recorded_data(self) -> Dict:
        return {"states": self.states if self.record_states else None,
                "actions": self.actions if self.record_actions else None,
                "contacts": self.contacts, "metadata": self.metadata}

    def reset(self):
        self.states: List[np.ndarray] = []
        self.actions: List[np.ndarray] = []
        self.contacts: List[List[float]] = []
        self.metadata: Dict = {}
