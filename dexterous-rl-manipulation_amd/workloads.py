"""BASELINE.json configs[1..4] as policy-gradient workloads (bench.py and the
full-size GPU parity tests build them here, so both run exactly the same thing).

  easy            C2  config_easy.json, 4096 envs/GPU
  default         C3  config_default.json: easy -> hard CurriculumScheduler
                      (experiments/config_default.json:16-23), fed every episode of
                      every rank (PGTrainer.attach_curriculum, dxrl_sched_scan)
  hard_heldout    C4  config_hard.json + HeldOutObjectSet(hard, n=10, seed=42)
                      (evaluation/heldout_objects.py:46-143), env i -> object i % 10, 8192 envs/GPU
  variable_noise  C5  config_variable.json + fused observation / dynamics noise 0.05
                      (robustness_tests.py:140-211; config_default.json:35-36 levels)

Episode success for the scheduler is ``success_rule="terminated"`` (>= 3 contacts, the
evaluators' rule, evaluator.py:157).  The reference's training loop reports success =
False for every episode (training/episode_utils.py:52), so under its
own rule the C3 scheduler never progresses; "terminated" is what makes C3 exercise it.
"""
from __future__ import annotations

from . import experiments
from .envs import VecEnv
from .experiments import CurriculumConfig

WORKLOADS = {
    "easy": {"config": "C2", "envs": 4096, "curriculum": "easy", "desc": "config_easy.json"},
    "default": {"config": "C3", "envs": 4096, "curriculum": "easy", "scheduler": True,
                "desc": "config_default.json (CurriculumScheduler easy->hard fed every finished episode of "
                        "every rank)"},
    "hard_heldout": {"config": "C4", "envs": 8192, "curriculum": "hard", "heldout": True,
                     "desc": "config_hard.json + HeldOutObjectSet table (env i -> object i % 10)"},
    "variable_noise": {"config": "C5", "envs": 4096, "curriculum": "variable", "obs_noise": 0.05,
                       "dyn_noise": 0.05, "desc": "config_variable.json + fused obs/dynamics noise 0.05"},
}

ENV_SEED = 20240601


def build_pg_workload(name: str, device, *, rank: int = 0, world: int = 1, process_group=None, envs=None,
                      horizon: int = 200, curriculum=None, seed: int = 7, scheduler_history: str = "window",
                      **trainer_kw):
    """(VecEnv, PGTrainer) for one rank of workload `name`; the env is reset."""
    from .trainer import PGTrainer, TrainerConfig
    w = WORKLOADS[name]
    n = envs or w["envs"]
    cur = curriculum or w["curriculum"]
    env = VecEnv(n, curriculum_config=CurriculumConfig.named(cur), reward_type="dense", seed=ENV_SEED,
                 device=device, global_env_offset=rank * n)
    if w.get("heldout"):
        from .evaluation import HeldOutObjectSet
        ex = experiments.load_named_config("default")
        hs = HeldOutObjectSet(CurriculumConfig.named(cur), num_heldout_objects=ex.evaluation.num_heldout_objects,
                              seed=ex.evaluation.seed)
        cfgs, idx = hs.native_table(n)
        env.set_curricula(cfgs, env_index=(idx + rank * n) % len(cfgs))
    kw = dict(horizon=horizon, seed=seed, obs_noise_std=w.get("obs_noise", 0.0), dyn_noise_std=w.get("dyn_noise", 0.0))
    kw.update(trainer_kw)
    tr = PGTrainer(env, TrainerConfig(**kw), process_group=process_group, world_size=world)
    if w.get("scheduler"):
        sc = experiments.load_named_config("default").curriculum_scheduler
        tr.attach_curriculum(experiments.CurriculumScheduler(
            CurriculumConfig.named(sc.initial_difficulty), CurriculumConfig.named(sc.target_difficulty),
            sc.success_rate_threshold, sc.min_episodes_before_progression, sc.window_size, sc.progression_steps,
            history=scheduler_history))
    env.reset(write_obs=False)
    return env, tr
