"""Golden fixtures for the evaluation drivers.

Run ONLY in the build container, after gen_golden.py's conditions hold:

    cd /tmp && python3 -B /root/repo/tests/golden/gen_eval_golden.py

Imports the reference read-only (through gen_golden's gymnasium stand-in) and
records what its evaluation drivers return:

* ``Evaluator.evaluate_heldout_set`` (evaluation/evaluator.py:183-262) with
  frozen SimpleLearner / HeuristicPolicy / RandomPolicy policies, the global
  np.random stream seeded once (exact reference order);
* ``Evaluator.evaluate_episode`` with np.random reseeded before every episode
  (the per-episode-stream form the vectorised evaluator runs in parallel);
* ``RobustnessTester.run_robustness_sweep`` / ``evaluate_with_noise``
  (evaluation/robustness_tests.py:240-407);
* ``EvaluationMetrics`` / ``format_metrics_report`` (evaluation/metrics.py)
  on synthetic episode lists, including the rounding ties of the failure rules.

Outputs (committed): tests/golden/eval_golden.json (inputs + expected outputs).
"""
import io
import json
import os
import sys
from contextlib import redirect_stdout

import numpy as np

sys.dont_write_bytecode = True
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden as G  # noqa: E402  (installs the stand-in, puts the reference on sys.path)

from envs import DexterousManipulationEnv  # noqa: E402
from evaluation.evaluator import Evaluator  # noqa: E402
from evaluation.heldout_objects import HeldOutObjectSet  # noqa: E402
from evaluation.metrics import EvaluationMetrics, format_metrics_report  # noqa: E402
from evaluation.robustness_tests import RobustnessTester  # noqa: E402
from policies.heuristic_policy import HeuristicPolicy  # noqa: E402
from policies.random_policy import RandomPolicy  # noqa: E402
from policies.simple_learner import SimpleLearner  # noqa: E402
from evaluation.failure_logger import FailureLogger  # noqa: E402
from evaluation.failure_taxonomy import FailureClassifier  # noqa: E402
from experiments.curriculum_logger import CurriculumLogger  # noqa: E402
from experiments.curriculum_scheduler import CurriculumScheduler  # noqa: E402
from experiments.config import CurriculumConfig  # noqa: E402
from training.logger import TrainingLogger  # noqa: E402
import tempfile  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def jsonable(x):
    if isinstance(x, dict):
        return {str(k): jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v) for v in x]
    if isinstance(x, (np.bool_, bool)):
        return bool(x)
    if isinstance(x, np.integer):
        return int(x)
    if isinstance(x, np.floating):
        return float(x)
    if isinstance(x, np.ndarray):
        return jsonable(x.tolist())
    return x


def episode_record(r):
    out = {k: r[k] for k in ("episode_reward", "episode_steps", "success", "num_contacts", "final_contacts")}
    out["contact_counts"] = [int(sum(1 for c in h if c > 0.5)) for h in r["contact_history"]]
    for k in ("object_size", "object_mass", "friction_coefficient", "object_idx", "episode"):
        if k in r:
            out[k] = r[k]
    return out


def make_policy(kind, mean, space_seed):
    space = DexterousManipulationEnv().action_space
    if kind == "simple":
        p = SimpleLearner(space)
        p.mean_action = np.asarray(mean, dtype=np.float32)
        return p
    if kind == "heuristic":
        return HeuristicPolicy(space)
    space.seed(space_seed)
    return RandomPolicy(space, seed=42)


MEANS = {
    "m1": [-0.3, -0.2, -0.1, 0.1, 0.2, 0.3, -0.4, -0.4, 0.0, 0.25, -0.25, 0.1, -0.1, 0.05, -0.05],
    "m2": [0.45, 0.4, 0.35, -0.45, -0.4, -0.35, 0.2, -0.2, 0.1, 0.0, 0.3, -0.3, 0.15, -0.15, 0.05],
    "zero": [0.0] * 15,
}

HELDOUT_CASES = [
    dict(name="simple_hard", policy="simple", mean="m1", np_seed=11, heldout=("hard", 10, 42), K=3, seed=100,
         reward="dense", max_steps=200),
    dict(name="heuristic_variable", policy="heuristic", mean="zero", np_seed=5, heldout=("variable", 4, 123), K=2,
         seed=5, reward="sparse", max_steps=60),
    dict(name="random_easy", policy="random", mean="zero", np_seed=0, space_seed=7, heldout=("easy", 5, 42), K=2,
         seed=0, reward="dense", max_steps=50),
    dict(name="simple_medium_m2", policy="simple", mean="m2", np_seed=23, heldout=("medium", 6, 7), K=4, seed=31,
         reward="dense", max_steps=120),
]

PER_EPISODE_CASES = [
    dict(name="per_episode_hard", policy="simple", mean="m2", heldout=("hard", 10, 42), K=4, seed=200,
         np_seed_base=1000, reward="dense", max_steps=200),
    dict(name="per_episode_heuristic", policy="heuristic", mean="zero", heldout=("variable", 5, 123), K=3, seed=7,
         np_seed_base=77, reward="dense", max_steps=100),
]

ROBUST_CASES = [
    dict(name="sweep_simple", kind="sweep", policy="simple", mean="m1", np_seed=3, cfg="variable", obs=[0.0, 0.05, 0.1],
         dyn=[0.0, 0.05, 0.1], episodes=3, seed=7, reward="dense", max_steps=80),
    dict(name="noise_heuristic", kind="single", policy="heuristic", mean="zero", np_seed=9, cfg="hard", obs_std=0.05,
         dyn_std=0.1, episodes=5, seed=9, reward="dense", max_steps=100),
    dict(name="sweep_random_sparse", kind="sweep", policy="random", mean="zero", np_seed=0, space_seed=3, cfg="easy",
         obs=[0.0, 0.02], dyn=[0.0, 0.2, 0.5], episodes=2, seed=1, reward="sparse", max_steps=40),
]


def gen_heldout(c):
    h = HeldOutObjectSet(G.make_cfg(c["heldout"][0]), num_heldout_objects=c["heldout"][1], seed=c["heldout"][2])
    pol = make_policy(c["policy"], MEANS[c["mean"]], c.get("space_seed"))
    np.random.seed(c["np_seed"])
    ev = Evaluator(pol, h, reward_type=c["reward"], max_episode_steps=c["max_steps"])
    res = ev.evaluate_heldout_set(num_episodes_per_object=c["K"], seed=c["seed"])
    after = np.random.standard_normal(3)
    after_space = pol.action_space.np_random.random(2) if c["policy"] == "random" else None
    return dict(c, episodes=[episode_record(r) for r in res["all_episodes"]], overall_stats=res["overall_stats"],
                metrics=res["metrics"], per_object_metrics=res["per_object_metrics"],
                per_object=[{k: v for k, v in o.items() if k != "episodes"} for o in res["per_object_results"].values()],
                report=format_metrics_report(res["metrics"]), np_random_after=after, space_random_after=after_space)


def gen_per_episode(c):
    h = HeldOutObjectSet(G.make_cfg(c["heldout"][0]), num_heldout_objects=c["heldout"][1], seed=c["heldout"][2])
    pol = make_policy(c["policy"], MEANS[c["mean"]], None)
    ev = Evaluator(pol, h, reward_type=c["reward"], max_episode_steps=c["max_steps"])
    eps = []
    for o in range(len(h.heldout_objects)):
        cfg = h.get_eval_config(o)
        for e in range(c["K"]):
            np.random.seed(c["np_seed_base"] + o * c["K"] + e)
            r = ev.evaluate_episode(cfg, seed=c["seed"] + e)
            r["object_idx"], r["episode"] = o, e
            eps.append(episode_record(r))
    return dict(c, episodes=eps)


def gen_robust(c):
    pol = make_policy(c["policy"], MEANS[c["mean"]], c.get("space_seed"))
    np.random.seed(c["np_seed"])
    rt = RobustnessTester(pol, G.make_cfg(c["cfg"]), reward_type=c["reward"], max_episode_steps=c["max_steps"])
    with redirect_stdout(io.StringIO()):
        if c["kind"] == "sweep":
            res = rt.run_robustness_sweep(c["obs"], c["dyn"], num_episodes=c["episodes"], seed=c["seed"])
        else:
            res = rt.evaluate_with_noise(c["obs_std"], c["dyn_std"], num_episodes=c["episodes"], seed=c["seed"])

    def one(r):
        return dict(episodes=[episode_record(e) for e in r["episodes"]], metrics=r["metrics"],
                    noise_levels=r["noise_levels"])

    if c["kind"] == "sweep":
        out = {"baseline": one(res["baseline"])}
        for grp in ("observation_noise", "dynamics_noise", "combined_noise"):
            out[grp] = [[str(k), one(v)] for k, v in res[grp].items()]
    else:
        out = one(res)
    return dict(c, result=out, np_random_after=np.random.standard_normal(3))


def metric_kats():
    """Synthetic episode lists through EvaluationMetrics (every failure rule and
    the f64 rounding ties of the variance / trend tests)."""
    rng = np.random.default_rng(2024)
    lists = []
    # the reference test's hand-made list (tests/test_evaluation_metrics.py:32-38)
    lists.append([
        {"success": True, "episode_steps": 50, "num_contacts": 4, "final_contacts": 4, "contact_history": []},
        {"success": True, "episode_steps": 75, "num_contacts": 5, "final_contacts": 5, "contact_history": []},
        {"success": False, "episode_steps": 200, "num_contacts": 2, "final_contacts": 2, "contact_history": []},
        {"success": False, "episode_steps": 150, "num_contacts": 1, "final_contacts": 0, "contact_history": []},
        {"success": True, "episode_steps": 30, "num_contacts": 3, "final_contacts": 3, "contact_history": []},
    ])

    def hist(counts):
        return [[1.0 if i < c else 0.0 for i in range(5)] for c in counts]

    ties = []
    # variance exactly 2.0 with an exact mean, and with non-integer means (searched)
    ties.append([0, 0, 2, 2, 2, 2, 4, 4])
    found = 0
    while found < 6:
        n = int(rng.integers(6, 40))
        c = rng.integers(0, 6, n)
        if n * int((c * c).sum()) - int(c.sum()) ** 2 == 2 * n * n and int(c.sum()) % n:
            ties.append(c.tolist())
            found += 1
    # trend exactly -1.0 (last5 - first5 sums differ by 5), low variance
    for f, l in [(8, 3), (6, 1), (5, 0), (10, 5), (9, 4), (7, 2)]:
        first = [f // 5 + (1 if i < f % 5 else 0) for i in range(5)]
        last = [l // 5 + (1 if i < l % 5 else 0) for i in range(5)]
        mid = [int(np.round((f + l) / 10))] * int(rng.integers(1, 6))
        ties.append(first + mid + last)
    eps = []
    for t in ties:
        eps.append({"success": False, "episode_steps": len(t), "num_contacts": t[-1], "final_contacts": t[-1],
                    "contact_history": hist(t)})
    lists.append(eps)
    # random episodes covering every branch
    eps = []
    for _ in range(300):
        n = int(rng.integers(1, 60))
        kind = rng.integers(0, 4)
        if kind == 0:
            c = rng.integers(0, 6, n)
        elif kind == 1:
            c = np.clip(np.linspace(int(rng.integers(2, 6)), int(rng.integers(0, 3)), n).round(), 0, 5).astype(int)
        elif kind == 2:
            c = np.full(n, int(rng.integers(0, 3)))
        else:
            c = rng.integers(1, 3, n)
        succ = bool(rng.random() < 0.3)
        steps = int(rng.choice([n, 60])) if not succ else n
        eps.append({"success": succ, "episode_steps": steps, "num_contacts": int(c[-1]),
                    "final_contacts": int(c[-1]), "contact_history": hist(c.tolist())})
    lists.append(eps)
    lists.append([eps[0]])  # single episode
    lists.append([e for e in eps if e["success"]][:5])  # no failures
    lists.append([e for e in eps if not e["success"]][:7])  # no successes
    out = []
    m = EvaluationMetrics(success_threshold=3)
    for L in lists:
        for max_steps in (60, 200):
            agg = m.compute_aggregate_metrics(L, max_steps=max_steps)
            per = [m.compute_episode_metrics(e, max_steps) for e in L]
            out.append(dict(max_steps=max_steps,
                            episodes=[{k: (v if k != "contact_history" else
                                           [int(sum(1 for x in h if x > 0.5)) for h in v]) for k, v in e.items()}
                                      for e in L],
                            aggregate=agg, per_episode=per,
                            report=format_metrics_report(agg) if agg else None))
    out.append(dict(max_steps=200, episodes=[], aggregate=m.compute_aggregate_metrics([], 200), per_episode=[],
                    report=None))
    return out


def gen_failure_log():
    """Evaluator + FailureLogger (evaluator.py:101-179): the logged entries minus timestamps."""
    c = HELDOUT_CASES[0]
    h = HeldOutObjectSet(G.make_cfg(c["heldout"][0]), num_heldout_objects=6, seed=c["heldout"][2])
    pol = make_policy(c["policy"], MEANS[c["mean"]], None)
    np.random.seed(c["np_seed"])
    with tempfile.TemporaryDirectory() as d:
        fl = FailureLogger(log_dir=d)
        ev = Evaluator(pol, h, reward_type="dense", max_episode_steps=9, failure_logger=fl)
        res = ev.evaluate_heldout_set(num_episodes_per_object=4, seed=c["seed"])
        entries = [{k: v for k, v in e.items() if k != "timestamp"} for e in fl.logged_episodes]
        stats = fl.get_statistics()
    return dict(policy=c["policy"], mean=c["mean"], np_seed=c["np_seed"], heldout=[c["heldout"][0], 6, c["heldout"][2]],
                K=4, seed=c["seed"], max_steps=9, entries=entries, statistics=stats,
                steps=[r["episode_steps"] for r in res["all_episodes"]])


def gen_taxonomy(metric_cases):
    clf = FailureClassifier(success_threshold=3)
    out = []
    for case in metric_cases:
        eps = [dict(e, contact_history=[[1.0 if i < c else 0.0 for i in range(5)] for c in e.get("contact_history", [])])
               for e in case["episodes"]]
        modes = [clf.classify(dict(e), case["max_steps"]) for e in eps]
        try:
            st = clf.get_failure_statistics([dict(e) for e in eps], case["max_steps"])
            st.pop("classified_episodes")
        except ZeroDivisionError:  # the reference divides by the episode count (failure_taxonomy.py:305)
            st = "ZeroDivisionError"
        out.append(dict(max_steps=case["max_steps"], episodes=case["episodes"],
                        modes=[[m.value if m else None, conf] for m, conf in modes], statistics=st))
    return out


def gen_training_logs():
    rng = np.random.default_rng(11)
    with tempfile.TemporaryDirectory() as d:
        tl = TrainingLogger(log_dir=d, experiment_name="kat")
        rewards = rng.normal(0.2, 0.4, 57).tolist()
        steps = rng.integers(1, 201, 57).tolist()
        succ = (rng.random(57) < 0.4).tolist()
        for k in range(57):
            tl.log_episode(k, rewards[k], int(steps[k]), bool(succ[k]),
                           reward_components={"distance": rewards[k] / 2} if k % 7 == 0 else None)
        path = tl.save()
        saved = json.load(open(path))
        stats3 = tl.get_statistics(window_size=3)
        sched = CurriculumScheduler(CurriculumConfig.easy(), CurriculumConfig.hard(), success_rate_threshold=0.3,
                                    window_size=10, min_episodes_before_progression=10, progression_steps=3)
        cl = CurriculumLogger(log_dir=d)
        cs = (rng.random(80) < 0.6).tolist()
        csteps = rng.integers(1, 201, 80).tolist()
        for k in range(80):
            prog = sched.update(bool(cs[k]), int(csteps[k]))
            cl.log_episode(k, sched, bool(cs[k]), int(csteps[k]))
            cl.log_progression(sched, prog)
        cpath = cl.save()
        csaved = json.load(open(cpath))
        buf = io.StringIO()
        with redirect_stdout(buf):
            cl.print_progression_summary(sched)
    return dict(rewards=rewards, steps=steps, success=succ, saved=saved, stats3=stats3,
                curriculum_success=cs, curriculum_steps=csteps, curriculum_saved=csaved, summary=buf.getvalue())


def gen_ablation():
    """train_with_config (evaluation/component_ablation.py:78-195) for the four ablation
    configurations x two seeds.  The reference seeds its env stream from OS entropy
    (env.reset() without a seed); for capture the stand-in's lazy seeding is pinned to
    env_seed, the value the build's train_with_config takes as its env_seed argument."""
    from evaluation.component_ablation import AblationConfig as RAC, train_with_config as rtwc
    from evaluation.component_ablation import compute_ablation_statistics as rstats
    orig = G._pcg
    runs, grouped = [], {}
    try:
        for name, cur, dense in [("baseline", True, True), ("no_curriculum", False, True),
                                 ("no_dense_reward", True, False), ("minimal", False, False)]:
            for seed, env_seed in [(42, 1001), (123, 1002)]:
                G._pcg = lambda s, es=env_seed: orig(es if s is None else s)
                r = rtwc(RAC(cur, dense, name), num_episodes=25, max_episode_steps=40, seed=seed)
                runs.append(dict(name=name, use_curriculum=cur, use_dense_reward=dense, seed=seed, env_seed=env_seed,
                                 result=r.to_dict(), np_random_after=np.random.standard_normal(2)))
                grouped.setdefault(name, []).append(r)
    finally:
        G._pcg = orig
    return dict(num_episodes=25, max_episode_steps=40, runs=runs, statistics=rstats(grouped))


class ObsPolicy:
    """A host policy the device kernel does not compile: deterministic, observation-dependent,
    f32 actions; update() counts calls (Evaluator must freeze it, evaluator.py:50-61)."""

    def __init__(self):
        self.W = np.random.default_rng(5).normal(0, 0.5, (15, 45))
        self.updates = 0

    def select_action(self, obs):
        return np.tanh(self.W @ np.asarray(obs, dtype=np.float64) + 0.3).astype(np.float32)

    def update(self, reward):
        self.updates += 1

    def reset(self):
        pass


def gen_host_policy():
    h = HeldOutObjectSet(G.make_cfg("easy"), num_heldout_objects=3, seed=123)
    pol = ObsPolicy()
    ev = Evaluator(pol, h, reward_type="dense", max_episode_steps=60)
    res = ev.evaluate_heldout_set(num_episodes_per_object=2, seed=7)
    rt = RobustnessTester(ObsPolicy(), G.make_cfg("variable"), reward_type="dense", max_episode_steps=50)
    rob = rt.evaluate_with_noise(0.05, 0.05, num_episodes=3, seed=3)
    return dict(episodes=[episode_record(r) for r in res["all_episodes"]], metrics=res["metrics"],
                updates=pol.updates, robustness=[episode_record(e) for e in rob["episodes"]],
                robustness_metrics=rob["metrics"])


def main():
    meta = {"generator": "tests/golden/gen_eval_golden.py", "numpy": np.__version__,
            "means": MEANS,
            "heldout": [gen_heldout(c) for c in HELDOUT_CASES],
            "per_episode": [gen_per_episode(c) for c in PER_EPISODE_CASES],
            "robustness": [gen_robust(c) for c in ROBUST_CASES],
            "metrics": metric_kats()}
    meta["taxonomy"] = gen_taxonomy(meta["metrics"])
    meta["failure_log"] = gen_failure_log()
    meta["training_logs"] = gen_training_logs()
    meta["ablation"] = gen_ablation()
    meta["host_policy"] = gen_host_policy()
    with open(os.path.join(OUT, "eval_golden.json"), "w") as f:
        json.dump(jsonable(meta), f, indent=None, separators=(",", ":"))
    print("wrote", os.path.join(OUT, "eval_golden.json"))


if __name__ == "__main__":
    main()
