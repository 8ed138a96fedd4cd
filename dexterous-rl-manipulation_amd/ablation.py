"""Component-ablation drivers -- evaluation/component_ablation.py:27-408 -- on the
fused SimpleLearner rollout (``dxrl_rollout_simple``).

``train_with_config`` is the reference's sequential loop: one env instance
(sticky object), one SimpleLearner carried across ``num_episodes``
``run_episode`` calls, the learner's np.random stream seeded with ``seed``.
Every (configuration, seed) run of ``run_component_ablation`` is one device
env lane, so the whole study is one launch sequence per reward type instead
of 4 x len(seeds) Python loops.  Each lane replays the reference's streams
exactly (training.ReferenceStreams): the legacy MT19937 gauss stream of
``np.random.seed(seed)`` and the env's gymnasium PCG64 stream.  The reference
seeds that env stream from OS entropy (``env.reset()`` without a seed), so
its runs are not repeatable; ``env_seed`` pins it (None = entropy, as there).

Quirk kept: run_episode reports success = info.get("success", False) = False
(episode_utils.py:52), so the CurriculumScheduler of a curriculum run never
progresses and every success rate is 0 -- the lane keeps the scheduler's
initial configuration, exactly as the reference does.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .envs import VecEnv
from .experiments import CurriculumConfig
from .policies import VecSimpleLearner
from .training import ReferenceStreams, SimpleLearnerRollout


@dataclass
class AblationConfig:
    """component_ablation.py:27-48."""
    use_curriculum: bool
    use_dense_reward: bool
    name: str = ""

    def __post_init__(self):
        if not self.name:
            self.name = "_".join(["curriculum" if self.use_curriculum else "no-curriculum",
                                  "dense-reward" if self.use_dense_reward else "sparse-reward"])


@dataclass
class TrainingResults:
    """component_ablation.py:51-75."""
    config: AblationConfig
    episode_rewards: List[float]
    episode_steps: List[int]
    success_rates: List[float]
    final_success_rate: float
    mean_episode_length: float
    convergence_step: Optional[int]
    total_episodes: int

    def to_dict(self) -> Dict:
        return {"config": asdict(self.config), "episode_rewards": self.episode_rewards,
                "episode_steps": self.episode_steps, "success_rates": self.success_rates,
                "final_success_rate": float(self.final_success_rate),
                "mean_episode_length": float(self.mean_episode_length),
                "convergence_step": self.convergence_step, "total_episodes": self.total_episodes}


_DIFFICULTY = {"easy": CurriculumConfig.easy, "medium": CurriculumConfig.medium, "hard": CurriculumConfig.hard}


def _lane_curriculum(cfg: AblationConfig, sched_cfg) -> CurriculumConfig:
    """component_ablation.py:97-140: a curriculum run starts (and, the scheduler never
    progressing, stays) at the scheduler's initial difficulty; otherwise the hard preset."""
    if not cfg.use_curriculum:
        return CurriculumConfig.hard()
    return _DIFFICULTY[sched_cfg.initial_difficulty if sched_cfg else "easy"]()


def _summarise(cfg: AblationConfig, rewards: np.ndarray, steps: np.ndarray, success: np.ndarray,
               num_episodes: int) -> TrainingResults:
    """component_ablation.py:168-186 (window-20 convergence, final rate over the last 20)."""
    rates = [1.0 if s else 0.0 for s in success]
    w = 20
    conv = None
    for i in range(w, len(rates)):
        if np.mean(rates[i - w:i]) >= 0.5:
            conv = i
            break
    final = np.mean(rates[-w:]) if len(rates) >= w else np.mean(rates)
    return TrainingResults(config=cfg, episode_rewards=[float(r) for r in rewards],
                           episode_steps=[int(s) for s in steps], success_rates=rates, final_success_rate=final,
                           mean_episode_length=np.mean([int(s) for s in steps]), convergence_step=conv,
                           total_episodes=num_episodes)


def _entropy_seed() -> int:
    return int(np.random.SeedSequence().entropy)


def train_many(jobs: Sequence[Tuple[AblationConfig, int]], num_episodes: int = 200, max_episode_steps: int = 200,
               learning_rate: float = 0.01, curriculum_scheduler_config=None,
               env_seeds: Optional[Sequence[Optional[int]]] = None, device=None,
               chunk_steps: int = 2048) -> Tuple[List[TrainingResults], List[int]]:
    """Every (configuration, seed) job as one env lane of fused rollouts (one env handle per
    reward type); returns the results in job order and the gauss draws each learner consumed."""
    if (curriculum_scheduler_config is not None and curriculum_scheduler_config.success_rate_threshold <= 0
            and any(c.use_curriculum for c, _ in jobs)):
        # with threshold <= 0 the reference's scheduler progresses even though training
        # episodes never report success (mean of an all-False window is 0.0 >= threshold,
        # component_ablation.py:160-170); the lanes here keep the initial difficulty
        raise ValueError("train_many assumes the ablation scheduler never progresses; "
                         "success_rate_threshold must be > 0")
    env_seeds = list(env_seeds) if env_seeds is not None else [None] * len(jobs)
    env_seeds = [_entropy_seed() if s is None else int(s) for s in env_seeds]
    results: List[Optional[TrainingResults]] = [None] * len(jobs)
    used = [0] * len(jobs)
    for dense in (True, False):
        lanes = [k for k, (c, _) in enumerate(jobs) if c.use_dense_reward == dense]
        if not lanes:
            continue
        n = len(lanes)
        env = VecEnv(n, reward_type="dense" if dense else "sparse", max_episode_steps=max_episode_steps,
                     device=device)
        idx = np.arange(n, dtype=np.int32)
        env.set_curricula([_lane_curriculum(jobs[k][0], curriculum_scheduler_config) for k in lanes], env_index=idx)
        learner = VecSimpleLearner(n, learning_rate=learning_rate, device=env.device)
        streams = ReferenceStreams(env, [env_seeds[k] for k in lanes], [jobs[k][1] for k in lanes])
        ro = SimpleLearnerRollout(env, learner, max_steps=max_episode_steps, record_cap=chunk_steps,
                                  success_rule="training", streams=streams)
        ro.start(env_index=idx)
        got: List[list] = [[] for _ in range(n)]
        remaining = np.full(n, int(num_episodes), dtype=np.int32)
        lane_used = np.zeros(n, dtype=np.int64)
        while remaining.max() > 0:
            rec = ro.run(chunk_steps, env_index=idx, episode_budget=torch.from_numpy(remaining).to(env.device))
            lane_used += ro.gauss_used.cpu().numpy()
            for j in np.lexsort((rec.end_step, rec.env_id)):  # per lane, in completion order
                got[int(rec.env_id[j])].append((rec.total_reward[j], rec.steps[j], rec.success[j]))
            counts = np.bincount(np.asarray(rec.env_id, dtype=np.int64), minlength=n)
            remaining = np.maximum(remaining - counts.astype(np.int32), 0)
        for li, k in enumerate(lanes):
            eps = got[li][:num_episodes]
            results[k] = _summarise(jobs[k][0], np.array([e[0] for e in eps], np.float64),
                                    np.array([e[1] for e in eps], np.int64), np.array([e[2] for e in eps], bool),
                                    num_episodes)
            used[k] = int(lane_used[li])
        env.close()
    return results, used


def train_with_config(config: AblationConfig, num_episodes: int = 200, max_episode_steps: int = 200,
                      seed: int = 42, learning_rate: float = 0.01, curriculum_scheduler_config=None,
                      env_seed: Optional[int] = None, device=None) -> TrainingResults:
    """component_ablation.py:78-195.  Leaves np.random where the reference leaves it:
    seeded with ``seed`` and advanced by the learner's draws."""
    (res,), (used,) = train_many([(config, seed)], num_episodes, max_episode_steps, learning_rate,
                                 curriculum_scheduler_config, [env_seed], device)
    np.random.seed(seed)
    np.random.standard_normal(used)
    return res


ABLATION_CONFIGS = [("baseline", True, True), ("no_curriculum", False, True), ("no_dense_reward", True, False),
                    ("minimal", False, False)]


def run_component_ablation(num_episodes: int = 200, max_episode_steps: int = 200, seeds: Optional[List[int]] = None,
                           learning_rate: float = 0.01, curriculum_scheduler_config=None, output_dir: str = "logs",
                           env_seeds: Optional[Dict[Tuple[str, int], int]] = None,
                           device=None) -> Dict[str, List[TrainingResults]]:
    """component_ablation.py:198-282: the four configurations x seeds as one batched run;
    results saved to <output_dir>/component_ablation_results.json."""
    seeds = [42, 123, 456] if seeds is None else list(seeds)
    configs = [AblationConfig(use_curriculum=c, use_dense_reward=d, name=nm) for nm, c, d in ABLATION_CONFIGS]
    jobs = [(c, s) for c in configs for s in seeds]
    es = [None if env_seeds is None else env_seeds.get((c.name, s)) for c, s in jobs]
    print("=" * 80)
    print("Component Ablation Study")
    print("=" * 80)
    print(f"Testing {len(configs)} configurations with {len(seeds)} seeds each")
    print(f"Episodes per run: {num_episodes}")
    print("=" * 80)
    flat, _ = train_many(jobs, num_episodes, max_episode_steps, learning_rate, curriculum_scheduler_config, es,
                         device)
    out: Dict[str, List[TrainingResults]] = {}
    for (c, _), r in zip(jobs, flat):
        out.setdefault(c.name, []).append(r)
    for c in configs:
        print(f"\nTesting: {c.name}")
        print(f"  Curriculum: {c.use_curriculum}")
        print(f"  Dense reward: {c.use_dense_reward}")
        for k, (s, r) in enumerate(zip(seeds, out[c.name])):
            print(f"  Seed {k + 1}/{len(seeds)} (seed={s})... Success rate: {r.final_success_rate:.3f}")
    os.makedirs(output_dir, exist_ok=True)
    path = Path(output_dir) / "component_ablation_results.json"
    with open(path, "w") as f:
        json.dump({k: [r.to_dict() for r in v] for k, v in out.items()}, f, indent=2)
    print(f"\nResults saved to: {path}")
    return out


def compute_ablation_statistics(all_results: Dict[str, List[TrainingResults]]) -> Dict[str, Dict]:
    """component_ablation.py:285-322."""
    stats = {}
    for name, rs in all_results.items():
        fsr = [r.final_success_rate for r in rs]
        mel = [r.mean_episode_length for r in rs]
        conv = [r.convergence_step for r in rs if r.convergence_step is not None]
        stats[name] = {
            "final_success_rate": {"mean": float(np.mean(fsr)), "std": float(np.std(fsr)),
                                   "min": float(np.min(fsr)), "max": float(np.max(fsr))},
            "mean_episode_length": {"mean": float(np.mean(mel)), "std": float(np.std(mel))},
            "convergence_step": {"mean": float(np.mean(conv)) if conv else None,
                                 "std": float(np.std(conv)) if conv else None, "num_converged": len(conv)},
        }
    return stats


def print_ablation_report(all_results: Dict[str, List[TrainingResults]], stats: Dict[str, Dict]):
    """component_ablation.py:325-408 (same text)."""
    bar, rule = "=" * 80, "-" * 80
    base_name = "baseline" if "baseline" in stats else list(stats)[0]
    base = stats[base_name]["final_success_rate"]["mean"]
    lines = ["\n" + bar, "Component Ablation Report", bar, "\nBaseline (Curriculum + Dense Reward):",
             f"  Final Success Rate: {base:.3f} +/- {stats[base_name]['final_success_rate']['std']:.3f}",
             "\n" + rule, "Component Contributions:", rule]
    for name, st in stats.items():
        if name == base_name:
            continue
        m, sd = st["final_success_rate"]["mean"], st["final_success_rate"]["std"]
        diff = m - base
        pct = (diff / base * 100) if base > 0 else 0
        lines += [f"\n{name.replace('_', ' ').title()}:", f"  Final Success Rate: {m:.3f} +/- {sd:.3f}",
                  f"  Difference from baseline: {diff:+.3f} ({pct:+.1f}%)"]
        c = st["convergence_step"]
        lines.append(f"  Convergence step: {c['mean']:.0f} +/- {c['std']:.0f}" if c["mean"] is not None
                     else "  Convergence: Not reached")
    lines += ["\n" + rule, "Key Insights:", rule]
    insights = [("no_curriculum", "Curriculum Learning Impact", "Without curriculum", "With curriculum", "Improvement"),
                ("no_dense_reward", "Dense Reward Impact", "Without dense reward", "With dense reward", "Improvement"),
                ("minimal", "Combined Impact", "Minimal (no curriculum, sparse reward)",
                 "Full system (curriculum + dense reward)", "Total improvement")]
    for k, (name, title, without, with_, label) in enumerate(insights, 1):
        if name not in stats:
            continue
        other = stats[name]["final_success_rate"]["mean"]
        d = base - other
        pct = (d / base * 100) if base > 0 else 0
        lines += [f"\n{k}. {title}:", f"   {without}: {other:.3f}", f"   {with_}: {base:.3f}",
                  f"   {label}: {d:+.3f} ({pct:+.1f}%)"]
    lines.append("\n" + bar)
    print("\n".join(lines))
