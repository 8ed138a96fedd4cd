"""Worker for tests/test_gpu_dist.py (not collected by pytest): one rank of a sharded
PGTrainer run on cuda:0.  Rank r owns envs [r*n, (r+1)*n) of a global batch (env /
policy streams keyed by global env id, as bench.py shards them), runs `iters` full
iterations (rollout, GAE with the global advantage moments, fused learner, gradient
all-reduce, Adam) and saves what the test compares against the world-1 run on the
concatenated batch.

    python tests/dist_pg_worker.py OUT.pt N_LOCAL ITERS CONFIG [MODE 0|1|u]   (RANK / WORLD_SIZE / MASTER_* in env)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out, n, iters, config, overlap="0"):
    import torch
    import dexterous_rl_manipulation_amd as pkg
    from dexterous_rl_manipulation_amd import distributed as D, envs, trainer
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # two ranks share the one GPU of a test box (RCCL refuses that)
        group = dist.group.WORLD
    cur = {"default": "easy"}.get(config, config)
    env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named(cur), reward_type="dense", seed=99,
                      device=dev, global_env_offset=rank * n)
    # overlap: "1" exchanges on the side stream (one fused call per network), "0" serialised with
    # the paired learner step (the default), "u" serialised, one call per network
    cfg = trainer.TrainerConfig(horizon=32, seed=4, ent_coef=0.01, max_steps=40,
                                record_cap=32 if config == "default" else 0, overlap_comm=overlap == "1",
                                pair_learner=overlap == "0")
    tr = trainer.PGTrainer(env, cfg, process_group=group, world_size=world)
    if config == "default":
        C = pkg.CurriculumConfig
        tr.attach_curriculum(pkg.experiments.CurriculumScheduler(C.easy(), C.hard(), 0.3, 20, 15, 5))
    env.reset(write_obs=False)
    first = None
    for k in range(iters):
        tr.iteration()
        if k == 0:
            first = (tr.grads.clone(), tr.rew.view(32, n).clone(), tr.done.view(32, n).clone(), tr.stats.clone())
    torch.cuda.synchronize()
    res = {"params": tr.params.cpu(), "grads0": first[0].cpu(), "rew0": first[1].cpu(), "done0": first[2].cpu(),
           "stats0": first[3].cpu(), "loss": tr.loss_stats()}
    if tr.scheduler is not None:
        res["sched"] = (tr.scheduler.total_episodes, tr.scheduler.total_steps, tr.scheduler.get_difficulty_level())
    torch.save(res, out)
    if world > 1:
        D.barrier(world, group)
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    run(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else "0")
