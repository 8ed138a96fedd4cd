"""CPU tests of the log formats and failure taxonomy against the
reference's outputs (tests/golden/eval_golden.json, made by gen_eval_golden.py)."""
import json

import numpy as np
import pytest

import dexterous_rl_manipulation_amd as pkg  # noqa: F401
from dexterous_rl_manipulation_amd import experiments as ex
from dexterous_rl_manipulation_amd import failures as F
from dexterous_rl_manipulation_amd import training as T
from dexterous_rl_manipulation_amd import evaluation as ev

from test_eval_host import golden, hist_dicts


@pytest.mark.parametrize("i", range(13))
def test_failure_classifier_matches_reference(i):
    case = golden()["taxonomy"][i]
    clf = F.FailureClassifier(success_threshold=3)
    eps = [dict(e, contact_history=hist_dicts(e.get("contact_history", []))) for e in case["episodes"]]
    got = [clf.classify(dict(e), case["max_steps"]) for e in eps]
    assert [[m.value if m else None, c] for m, c in got] == case["modes"]
    if case["statistics"] == "ZeroDivisionError":
        with pytest.raises(ZeroDivisionError):
            clf.get_failure_statistics([dict(e) for e in eps], case["max_steps"])
    else:
        st = clf.get_failure_statistics([dict(e) for e in eps], case["max_steps"])
        st.pop("classified_episodes")
        assert st == case["statistics"]


def test_failure_mode_definitions_surface():
    assert [m.value for m in F.FailureMode] == ["slippage", "unstable_grasp", "misalignment", "timeout",
                                                "object_dropped", "insufficient_contacts"]
    d = F.FAILURE_MODE_DEFINITIONS
    assert d[F.FailureMode.SLIPPAGE].detection_criteria["contact_trend_threshold"] == -1.0
    assert d[F.FailureMode.UNSTABLE_GRASP].detection_criteria["contact_variance_threshold"] == 2.0
    assert ev.FailureClassifier is F.FailureClassifier and ev.FailureLogger is F.FailureLogger


def test_training_logger_matches_reference(tmp_path):
    g = golden()["training_logs"]
    tl = T.TrainingLogger(log_dir=str(tmp_path), experiment_name="kat")
    for k, (r, s, ok) in enumerate(zip(g["rewards"], g["steps"], g["success"])):
        tl.log_episode(k, r, int(s), bool(ok), reward_components={"distance": r / 2} if k % 7 == 0 else None)
    assert json.load(open(tl.save())) == g["saved"]
    assert tl.get_statistics(window_size=3) == g["stats3"]
    # device-record ingestion builds the same series
    rec = T.EpisodeRecords(env_id=np.zeros(57, np.int64), end_step=np.arange(57), total_reward=np.array(g["rewards"]),
                           steps=np.array(g["steps"], np.int32), success=np.array(g["success"]))
    tl2 = T.TrainingLogger(log_dir=str(tmp_path), experiment_name="kat2")
    tl2.log_records(rec)
    assert tl2.episode_rewards == tl.episode_rewards and tl2.episode_steps == tl.episode_steps
    assert tl2.success_rates == tl.success_rates and tl2.convergence_step == tl.convergence_step
    assert tl2.get_statistics() == tl.get_statistics()


def test_curriculum_logger_matches_reference(tmp_path, capsys):
    g = golden()["training_logs"]
    sched = ex.CurriculumScheduler(ex.CurriculumConfig.easy(), ex.CurriculumConfig.hard(), success_rate_threshold=0.3,
                                   window_size=10, min_episodes_before_progression=10, progression_steps=3)
    cl = ex.CurriculumLogger(log_dir=str(tmp_path))
    for k, (ok, st) in enumerate(zip(g["curriculum_success"], g["curriculum_steps"])):
        prog = sched.update(bool(ok), int(st))
        cl.log_episode(k, sched, bool(ok), int(st))
        cl.log_progression(sched, prog)
    assert json.load(open(cl.save())) == g["curriculum_saved"]
    cl.print_progression_summary(sched)
    assert capsys.readouterr().out == g["summary"]


def test_failure_logger_roundtrip(tmp_path):
    fl = F.FailureLogger(log_dir=str(tmp_path))
    ep = {"success": False, "episode_steps": 12, "episode_reward": 1.5, "num_contacts": 2, "final_contacts": 2,
          "contact_history": hist_dicts([2] * 12), "object_size": 0.05}
    e = fl.log_episode(ep, states=[np.zeros(45, np.float32)] * 13, actions=[np.ones(15, np.float32)] * 12,
                       metadata={"seed": np.int64(3)}, max_steps=200)
    assert e["failure_mode"] == "misalignment" and e["failure_confidence"] == {"misalignment": 0.8}
    path = fl.save("f.json")
    fl2 = F.FailureLogger(log_dir=str(tmp_path))
    data = fl2.load(str(path))
    assert data["metadata"]["failure_modes"] == {"misalignment": 1} and fl2.episode_counter == 1
    assert fl2.logged_episodes[0]["metadata"] == {"seed": 3} and len(fl2.logged_episodes[0]["states"]) == 13
    assert fl2.get_statistics()["mean_episode_length"] == 12.0
    r = F.EpisodeRecorder()
    r.record_step(state=np.zeros(3), contacts=[1, 0])
    r.set_metadata(seed=1)
    assert r.get_recorded_data()["contacts"] == [[1.0, 0.0]]


def test_ablation_config_and_statistics_match_reference():
    """AblationConfig naming (reference tests/test_component_ablation.py:25-38) and
    compute_ablation_statistics over the reference's own results."""
    from dexterous_rl_manipulation_amd import ablation as A
    assert A.AblationConfig(True, True).name == "curriculum_dense-reward"
    assert A.AblationConfig(False, False).name == "no-curriculum_sparse-reward"
    assert A.AblationConfig(True, False, name="custom").name == "custom"
    g = golden()["ablation"]
    grouped = {}
    for r in g["runs"]:
        d = r["result"]
        cfg = A.AblationConfig(**d["config"])
        grouped.setdefault(r["name"], []).append(A.TrainingResults(
            cfg, d["episode_rewards"], d["episode_steps"], d["success_rates"], d["final_success_rate"],
            d["mean_episode_length"], d["convergence_step"], d["total_episodes"]))
        summ = A._summarise(cfg, np.array(d["episode_rewards"]), np.array(d["episode_steps"]),
                            np.array(d["success_rates"]) > 0.5, d["total_episodes"])
        assert summ.to_dict() == d
    assert A.compute_ablation_statistics(grouped) == g["statistics"]
