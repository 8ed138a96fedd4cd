"""dexterous-rl-manipulation_amd -- MI355X-native hot path of I2S9/dexterous-rl-manipulation.

Drop-in surfaces (same names as the reference modules):
  envs.DexterousManipulationEnv, rewards.{RewardShaping,SparseReward},
  policies.{SimpleLearner,RandomPolicy,HeuristicPolicy}, training.{run_episode,run_training_episode},
  experiments.{CurriculumConfig,CurriculumScheduler,StepBasedScheduler,ExperimentConfig,load_config,...},
  evaluation.{HeldOutObjectSet,CombinedNoiseWrapper,Evaluator,RobustnessTester,EvaluationMetrics,...}
Batched device API: envs.VecEnv, policies.VecSimpleLearner, training.SimpleLearnerRollout.
The compute runs in libdxrl.so (HIP, gfx950; C ABI in include/dxrl.h).  No CPU fallback.
"""
from . import experiments, rewards  # noqa: F401  (no GPU needed to import)
from .experiments import CurriculumConfig  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    import importlib
    if name in ("envs", "policies", "training", "evaluation", "build", "_native", "trainer",
                "evaluator", "metrics"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
