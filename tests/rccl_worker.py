"""Worker for tests/test_gpu_rccl.py (not collected by pytest): a world-1 RCCL process group
(backend "nccl" = RCCL on ROCm, bound to cuda:0 with device_id) executes every collective the
sharded PG trainer makes -- through distributed.py, with the same calls a multi-rank job
issues -- and a PGTrainer given that group must produce exactly what the group-less world-1
trainer produces.

    python tests/rccl_worker.py OUT.pt      (MASTER_ADDR / MASTER_PORT in env)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trainer_run(pkg, group, n, iters, config, dev, overlap=True, updates=None, reserve_cus=0, pair=None):
    from dexterous_rl_manipulation_amd import envs, trainer
    cur = {"default": "easy"}.get(config, config)
    env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named(cur), reward_type="dense", seed=99,
                      device=dev)
    cfg = trainer.TrainerConfig(horizon=32, seed=4, ent_coef=0.01, max_steps=40,
                                obs_noise_std=0.05 if config == "variable" else 0.0,
                                dyn_noise_std=0.05 if config == "variable" else 0.0, overlap_comm=overlap,
                                reserve_cus=reserve_cus, pair_learner=(not overlap) if pair is None else pair)
    tr = trainer.PGTrainer(env, cfg, process_group=group, world_size=1)
    if config == "default":
        C = pkg.CurriculumConfig
        tr.attach_curriculum(pkg.experiments.CurriculumScheduler(C.easy(), C.hard(), 0.3, 20, 15, 5))
    env.reset(write_obs=False)
    out = {"grads": [], "stats": [], "codes": []}
    for k in range(iters):
        tr.iteration(update=True if updates is None else updates[k])
        out["grads"].append(tr.grads.cpu().clone())
        out["stats"].append(tr.stats.cpu().clone())
        if tr.scheduler is not None:
            out["codes"].append(tr.ep_code.cpu().clone())
    import torch
    torch.cuda.synchronize()
    out["params"] = tr.params.cpu()
    out["collective"] = tr.collective
    out["overlapped"] = tr._comm is not None
    if tr.scheduler is not None:
        out["sched"] = (tr.scheduler.total_episodes, tr.scheduler.total_steps, tr.scheduler.get_difficulty_level())
    return out


def run(out_path):
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    g = dist.group.WORLD
    import dexterous_rl_manipulation_amd as pkg
    from dexterous_rl_manipulation_amd import distributed as D, trainer
    res = {"backend": dist.get_backend(g)}
    gen = torch.Generator(device="cpu").manual_seed(0)
    # the trainer's exchanges, one by one (trainer.py optimizer_step / advantages / schedule_feed)
    grads = torch.randn(trainer.NPARAMS, generator=gen).to(dev)
    x = grads.clone()
    D.all_reduce_sum_(x, 1, g)
    res["allreduce_equal"] = bool(torch.equal(x, grads))
    stats = torch.randn(8, dtype=torch.float64, generator=gen).to(dev)
    mom = torch.zeros(1, 3, dtype=torch.float64, device=dev)
    D.gather_adv_moments_(mom, stats, 1, g)
    res["moments_equal"] = bool(torch.equal(mom[0], stats[5:8]))
    codes = torch.randint(-32768, 32767, (32 * 256,), dtype=torch.int16, generator=gen).to(dev)
    codes_all = torch.zeros_like(codes)
    D.all_gather_into_(codes_all, codes, 1, g)
    res["codes_equal"] = bool(torch.equal(codes_all, codes))
    res["global_count"] = D.global_count(12345, 1, g)
    res["max"] = D.all_reduce_max(3.25, 1, dev, g)
    D.barrier(1, g)
    # the whole trainer through the RCCL group vs without any group
    for config in ("default", "variable"):
        # exchanges on the side stream (default), no group, exchanges serialised on the compute stream
        # overlapped through the group, no group, serialised through the group (both with one learner
        # call per network, the form the overlapped exchanges need), serialised + paired through the
        # group == paired without a group (the default trainer)
        res[config] = (trainer_run(pkg, g, 256, 3, config, dev), trainer_run(pkg, None, 256, 3, config, dev, pair=False),
                       trainer_run(pkg, g, 256, 3, config, dev, overlap=False, pair=False))
        res[config + "_paired"] = (trainer_run(pkg, g, 256, 3, config, dev, overlap=False),
                                   trainer_run(pkg, None, 256, 3, config, dev, overlap=False))
        # an iteration without the optimiser step between two with it: the overlapped form issues
        # no gradient collective there and leaves nothing in flight (== no group, bit for bit)
        upd = (True, False, True, True)
        res[config + "_noupdate"] = (trainer_run(pkg, g, 256, 4, config, dev, updates=upd),
                                     trainer_run(pkg, None, 256, 4, config, dev, updates=upd, pair=False))
        # CUs reserved for the collectives: overlapped == serialised at the same reservation
        res[config + "_reserve"] = (trainer_run(pkg, g, 256, 3, config, dev, reserve_cus=4),
                                    trainer_run(pkg, g, 256, 3, config, dev, overlap=False, reserve_cus=4, pair=False))
    torch.save(res, out_path)
    dist.destroy_process_group()


if __name__ == "__main__":
    run(sys.argv[1])
