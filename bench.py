"""Benchmark: env-steps/sec of the vectorised rollout hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--horizon 200]

One bench "step" = one training iteration of the hot path over one batch
(BASELINE configs[1]: config_easy curriculum, dense reward, 4096 envs per
GPU, MLP(256,256) learner, synthetic device-Philox randomness):

  --learner pg (default): PGTrainer.iteration() -- every env advances
      `horizon` env steps with the actor MLP fused into the step kernel, then
      critic forward, GAE, advantage normalisation, PPO heads, backward GEMMs,
      gradient all-reduce (RCCL, world > 1) and Adam.
  --learner simple: the reference's run_episode + SimpleLearner loop
      (training/episode_utils.py:13-55, policies/simple_learner.py) for
      `horizon` steps per env, fused into one HIP launch.

Multi-GPU, one rank per GPU over RCCL: either the driver's
`torchrun --nproc-per-node N bench.py --gpus N`, or plain `bench.py --gpus N`,
which starts that torchrun command as a child process before anything touches
the GPU (and refuses when fewer than N GPUs are visible).  Env shards are
independent (global env ids rank*N .. rank*N+N-1); the PG learner all-reduces
the advantage moments and one flat f32 gradient buffer per iteration; the
timing uses a barrier + max-over-ranks.  value = all ranks' env steps / max
time (weak scaling).

Also measured in-process (HIP events on the launch stream):
  * roofline: the standalone step kernel (dxrl_env_step, k_step) at a large N
    (default 2^22 envs, traffic >> the 256 MB Infinity Cache) -- the
    "%HBM roofline step kernel" half of the BASELINE metric;
  * cpu_baseline: the CPU oracle's run_episode + SimpleLearner loop (the
    reference's algorithm restated), one core, a bounded ~10 s sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# oracle loop / the reference's own loop, same core, build container (tools/cpu_ratio.py)
RESTATEMENT_SPEED_RATIO = {"easy": 1.26, "hard": 0.96}
STEP_BYTES_PER_ENV = 594  # k_step algorithmic bytes per env-step


# BASELINE.json configs[1..4] as PG workloads (configs[0] is the CPU plumbing case)
_PKG = os.path.join(ROOT, "dexterous-rl-manipulation_amd")
sys.path.insert(0, ROOT)
import dexterous_rl_manipulation_amd  # noqa: E402,F401  (the package alias)
from dexterous_rl_manipulation_amd.workloads import WORKLOADS, build_pg_workload  # noqa: E402


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--prewarm-s", type=float, default=2.0,
                   help="untimed iterations for at least this long before the --warmup ones: the GPU's clocks "
                        "take the first ~1-2 s of work to reach their sustained level (DESIGN.md §6)")
    p.add_argument("--config", choices=sorted(WORKLOADS), default="easy",
                   help="BASELINE configs[1..4]: easy (C2, the metric's config), default (C3: curriculum "
                        "scheduler), hard_heldout (C4: held-out object table, 8192 envs), variable_noise (C5)")
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's)")
    p.add_argument("--horizon", type=int, default=200, help="env steps per bench step (rollout length)")
    p.add_argument("--curriculum", default=None, help="override the config's curriculum preset")
    p.add_argument("--epochs", type=int, default=1, help="PPO epochs per iteration (default 1: A2C-style step)")
    p.add_argument("--minibatches", type=int, default=1, help="PPO minibatches per epoch")
    p.add_argument("--learner", choices=["pg", "simple"], default="pg",
                   help="pg: MLP actor-critic policy-gradient iteration (default); simple: SimpleLearner rollout")
    p.add_argument("--roofline-envs", type=int, default=1 << 22)
    p.add_argument("--roofline-launches", type=int, default=30)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--success-rule", choices=["terminated", "training"], default=None,
                   help="episode success for the C3 scheduler: terminated (the evaluators' rule, default) or "
                        "training (the reference's training loop: always False, so it never progresses)")
    p.add_argument("--sched-restart", action="store_true",
                   help="C3: restart the CurriculumScheduler from its initial config at the start of every "
                        "iteration (CurriculumScheduler.reset()), so every timed iteration replays progressions")
    p.add_argument("--overlap", action="store_true",
                   help="exchanges on a side stream beside the train passes (TrainerConfig.overlap_comm=True; "
                        "default: serialised on the compute stream, DESIGN.md §7)")
    p.add_argument("--recompute-h2", action="store_true",
                   help="A/B: the first train pass of an iteration recomputes layer 2 instead of reading the "
                        "activations the rollout / critic-values pass stored (TrainerConfig.reuse_h2=False)")
    p.add_argument("--reserve-cus", type=int, default=0,
                   help="CUs kept free of the persistent learner kernels for the side-stream collectives "
                        "(TrainerConfig.reserve_cus)")
    p.add_argument("--dist", action="store_true",
                   help="create the RCCL process group even at --gpus 1 (before any GPU work) and run the "
                        "multi-rank code path: the trainer's collectives, barrier and max-over-ranks timing")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="process-group backend: nccl (RCCL over xGMI, one rank per GPU: the driver's scaling "
                        "runs) or gloo (host-staged exchanges; ranks may share a GPU, rank r on GPU r mod the "
                        "visible count -- exercises the multi-rank harness on a one-GPU box, not a scaling "
                        "measurement)")
    a = p.parse_args()
    w = WORKLOADS[a.config]
    a.envs = a.envs or w["envs"]
    a.curriculum = a.curriculum or w["curriculum"]
    return a


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without torchrun: start N ranks (torch.distributed.run, one process
    per GPU, rendezvous on 127.0.0.1) as a child process and return its exit code.  Called
    before this process initialises the GPU (device_count() does not, on ROCm)."""
    import socket
    import subprocess
    have = torch.cuda.device_count()
    if have < (1 if args.backend == "gloo" else args.gpus):
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {have}", file=sys.stderr)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    """One rank per GPU over RCCL (torch.distributed "nccl").  With --dist a world-1 process
    group is created too, so the collectives run exactly as in a multi-rank job.  --backend gloo:
    rank r runs on GPU r mod the visible count (ranks may share one).  Returns (world, rank,
    device index)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    if world > 1 or args.dist:
        import socket
        import torch.distributed as dist
        if "MASTER_PORT" not in os.environ:  # plain `bench.py --dist` (no torchrun)
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
            s.close()
        torch.cuda.set_device(local)
        if args.backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(world):
    if _dist_on():
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world, dev):
    if not _dist_on():
        return x
    import torch.distributed as dist
    gloo = dist.get_backend() == "gloo"  # gloo reduces host tensors
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if gloo else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# Algorithmic FLOPs per env-step (unpadded 45->256->256->{15,1} shapes):
FWD_ACTOR = 2 * (45 * 256 + 256 * 256 + 256 * 15)      # 161,792 (rollout policy, per env step)
FWD_BOTH = FWD_ACTOR + 2 * (45 * 256 + 256 * 256 + 256)  # 316,416 (training forward, both nets)
BWD_BOTH = FWD_BOTH + 2 * (256 * 256 + 256 * 15) + 2 * (256 * 256 + 256)  # weight + input grads
PEAK_BF16_TFS = 2500.0  # dense bf16 MFMA peak (MI355X_MICROARCH.md)


def pg_bench(args, world, rank, dev):
    """One bench step = one PGTrainer.iteration(): rollout (T env steps of every env, actor
    MLP fused) + critic forward + GAE + adv-norm + actor forward + heads + backward +
    RCCL gradient all-reduce (world > 1) + Adam."""
    pg = None
    if _dist_on():  # world > 1, or --dist: the trainer runs its collectives over RCCL
        import torch.distributed as dist
        pg = dist.group.WORLD
    kw = {"success_rule": args.success_rule} if args.success_rule else {}
    if args.overlap:
        kw["overlap_comm"] = True
    if args.reserve_cus:
        kw["reserve_cus"] = args.reserve_cus
    if args.recompute_h2:
        kw["reuse_h2"] = False
    env, tr = build_pg_workload(args.config, dev, rank=rank, world=world, process_group=pg, envs=args.envs,
                                horizon=args.horizon, curriculum=args.curriculum, epochs=args.epochs,
                                minibatches=args.minibatches, **kw)
    sc = tr.scheduler
    if args.sched_restart and sc is None:
        raise SystemExit("--sched-restart needs a workload with a curriculum scheduler (--config default)")

    def one_iteration():
        if args.sched_restart:  # a fresh scheduler: level 0, empty window, the initial config on the device
            sc.reset()
            env.set_curriculum_async(sc.get_current_config())
        tr.iteration()

    # bring the GPU to its sustained clock first (not part of the W warmup steps or the timed K):
    # blocks of 8 iterations until the slowest rank has run for prewarm_s (every rank runs the
    # same number of iterations, so their collectives pair up)
    prewarm_iters, tp, prewarm_s = 0, time.perf_counter(), 0.0
    while prewarm_s < args.prewarm_s:
        for _ in range(8):
            one_iteration()
        torch.cuda.synchronize(dev)
        prewarm_iters += 8
        prewarm_s = max_over_ranks(time.perf_counter() - tp, world, dev)
    for _ in range(args.warmup):
        one_iteration()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    prog0 = len(sc.progression_history) if sc is not None else 0
    prog_timed = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if args.sched_restart:
            prog0 = 0
        one_iteration()
        if sc is not None:  # host list length: no device work, no sync
            prog_timed += len(sc.progression_history) - prog0
            prog0 = len(sc.progression_history)
    torch.cuda.synchronize(dev)
    barrier(world)
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, world, dev)
    # phase breakdown (one extra iteration, outside the timed region)
    stream = torch.cuda.current_stream(dev)
    names = tr.phases()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
    evs[0].record(stream)
    for k, nm in enumerate(names):
        getattr(tr, nm)()
        evs[k + 1].record(stream)
    torch.cuda.synchronize(dev)
    phases = {nm: round(evs[k].elapsed_time(evs[k + 1]), 4) for k, nm in enumerate(names)}
    M = tr.M
    gemm_ms = sum(v for k, v in phases.items() if k not in ("rollout", "advantages", "optimizer_step",
                                                            "schedule_feed", "schedule_apply"))
    train_flops = M * args.epochs * (FWD_BOTH + BWD_BOTH)
    # (reuse_h2: the first train pass reads the actor's layer 2 from the rollout's tape -- computed in
    # the rollout phase, outside gemm_ms -- so that pass's share of it is not counted here; the
    # critic's comes from the critic-values pass, inside gemm_ms)
    l2_from_rollout = M * 2 * 256 * 256 if getattr(tr, "h2a_tape_written", False) else 0
    train_flops -= l2_from_rollout
    mfma = {"bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_BF16_TFS,
            "training_gemms_achieved": round(train_flops / (gemm_ms * 1e-3) / 1e12, 2),
            "rollout_policy_achieved": round(M * FWD_ACTOR / (phases["rollout"] * 1e-3) / 1e12, 2),
            "algorithmic_flop_per_env_step": {"rollout_actor_fwd": FWD_ACTOR, "train_fwd": FWD_BOTH,
                                              "train_bwd": BWD_BOTH},
            "train_l2_read_from_rollout_flop": l2_from_rollout}
    mfma["frac"] = round(mfma["training_gemms_achieved"] / PEAK_BF16_TFS, 4)
    stats = tr.episode_stats()
    if tr.scheduler is not None:
        stats["curriculum_level"] = tr.scheduler.get_difficulty_level()
        stats["scheduler_episodes"] = int(tr.scheduler.total_episodes)
        stats["progressions_applied_in_timed_iterations"] = prog_timed
        stats["success_rule"] = tr.cfg.success_rule
    stats["prewarm"] = {"s": round(prewarm_s, 3), "iterations": prewarm_iters}
    stats.update({k: round(v, 5) for k, v in tr.loss_stats().items()})
    return wall, phases, mfma, stats


def rollout_bench(args, world, rank, dev):
    import dexterous_rl_manipulation_amd as pkg
    from dexterous_rl_manipulation_amd import envs, policies, training
    n = args.envs
    env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.named(args.curriculum), reward_type="dense",
                      seed=20240601, device=dev, global_env_offset=rank * n)
    learner = policies.VecSimpleLearner(n, seed=777, device=dev)
    ro = training.SimpleLearnerRollout(env, learner)
    ro.start()
    for _ in range(args.warmup):
        ro.run(args.horizon, collect=False)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        ro.run(args.horizon, collect=False)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    wall = max_over_ranks(wall, world, dev)
    # bookkeeping check outside the timed region
    rec = ro.run(args.horizon)
    assert rec.dropped == 0 and len(rec) > 0
    return wall, kernel_ms


def step_kernel_time(n, launches, dev, seed=5):
    """k_step (dxrl_env_step) on n envs: HIP events around `launches` back-to-back launches on
    the launch stream; ms per launch (synthetic U(-1.2, 1.2) actions, variable curriculum)."""
    from dexterous_rl_manipulation_amd import envs
    import dexterous_rl_manipulation_amd as pkg
    env = envs.VecEnv(n, curriculum_config=pkg.CurriculumConfig.variable(), reward_type="dense", seed=seed,
                      device=dev)
    env.reset(write_obs=False)
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    acts = (torch.rand(n, 15, generator=gen, device=dev) * 2.4 - 1.2).contiguous()
    for _ in range(3):
        env.step(acts)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)  # dxrl_env_step launches on this stream
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(launches):
        env.step(acts)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    ms = ev0.elapsed_time(ev1) / launches
    del env, acts
    torch.cuda.empty_cache()
    return ms


def step_kernel_small(n, dev):
    """The BASELINE.md "step-kernel env-steps/s @4096" column: k_step at the bench's env count
    (cache-resident, launch-latency bound; not a roofline figure)."""
    ms = step_kernel_time(n, 200, dev)
    return {"envs": n, "us_per_launch": round(ms * 1e3, 2), "env_steps_per_s": round(n / (ms * 1e-3), 1),
            "algorithmic_GB_s": round(STEP_BYTES_PER_ENV * n / (ms * 1e-3) / 1e9, 1),
            "note": "back-to-back launches, HIP events; working set in L2 / Infinity Cache"}


def step_kernel_roofline(args, dev):
    """k_step at large N: algorithmic bytes / HIP-event time per launch."""
    n = args.roofline_envs
    ms = step_kernel_time(n, args.roofline_launches, dev)
    # traffic: PMC-corrected HBM bytes per launch (2 FETCH_SIZE + WRITE_SIZE, separate --pmc passes,
    # tools/profile_round.sh) from the newest round's profiles/rNN/pmc_step_kernel.json
    traffic, src = None, None
    import glob
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "pmc_step_kernel.json")), reverse=True):
        with open(pmc) as f:
            d = json.load(f)
        if d.get("envs") == n:
            traffic, src = d.get("hbm_bytes_per_launch"), os.path.relpath(pmc, ROOT)
            break
    bytes_per_launch = STEP_BYTES_PER_ENV * n
    achieved = bytes_per_launch / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": src,
            "traffic_per_algorithmic_byte": round(traffic / bytes_per_launch, 4) if traffic else None,
            "kernel": "k_step (dxrl_env_step)",
            "envs": n, "bytes_per_env_step": STEP_BYTES_PER_ENV, "ms_per_launch": round(ms, 4),
            "env_steps_per_s": round(n / (ms * 1e-3), 1)}


def _cpu_worker(curriculum, seconds, seed, out):
    """One host core: the reference's run_episode + SimpleLearner loop over the oracle env
    (training/episode_utils.py:13-55, policies/simple_learner.py:49-99), 1 env."""
    from oracle.dx_oracle import OracleCurriculum, OracleEnv, OracleSimpleLearner, reset_draws
    presets = {"easy": dict(object_size=0.08, object_mass=0.05, friction_coefficient=0.8),
               "medium": {}, "hard": dict(object_size=0.03, object_mass=0.2, friction_coefficient=0.3),
               "variable": dict(size_range=(0.03, 0.07), mass_range=(0.05, 0.15), friction_range=(0.3, 0.7))}
    cur = OracleCurriculum(**presets.get(curriculum, {}))
    env = OracleEnv(cur=cur, dense=True)
    pol = OracleSimpleLearner(np.random.RandomState(42 + seed).standard_normal(4_000_000), learning_rate=0.01)
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(1000 + seed)))
    steps, first = 0, True
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and pol.cur < 3_900_000:
        env.reset(reset_draws(rng, cur, first))
        first = False
        pol.reset()
        for _ in range(200):
            a = pol.select_action()
            _, r, te, tr = env.step(a)
            pol.update(r)
            steps += 1
            if te or tr:
                break
    out.put((steps, time.perf_counter() - t0))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args):
    """The reference algorithm restated (oracle/dx_oracle.py) in the reference's own loop shape,
    1 env per process: P = 1 and P = every host core this job may use (the
    affinity mask, at most 16 -- the box's CPU share per GPU), `--cpu-seconds` each.  Runs
    before this process touches the GPU; workers are spawned interpreters."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    p_all = max(1, min(avail, 16))
    res = {}
    for P in sorted({1, p_all}):
        q = ctx.Queue()
        procs = [ctx.Process(target=_cpu_worker, args=(args.curriculum, args.cpu_seconds, k, q)) for k in range(P)]
        for pr in procs:
            pr.start()
        got = [q.get(timeout=args.cpu_seconds + 120) for _ in procs]
        for pr in procs:
            pr.join()
        res[P] = (sum(st for st, _ in got), sum(st / dt for st, dt in got))
    steps1, v1 = res[1]
    stepsP, vP = res[p_all]
    return {"value": round(vP, 1), "unit": "env-steps/s", "cores": p_all, "kind": "port",
            "single_core": round(v1, 1), "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"oracle/dx_oracle.py run_episode+SimpleLearner loop (the reference's loop restated), "
                      f"config_{args.curriculum}, 1 env per process, {args.cpu_seconds:.0f} s per run: "
                      f"P=1 {steps1} env-steps, P={p_all} {stepsP} env-steps (aggregate of per-process rates); "
                      f"the restatement runs at {RESTATEMENT_SPEED_RATIO} x the reference's own loop speed on one "
                      f"core (tools/cpu_ratio.py, DESIGN.md §6)"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    cpu = None
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)  # before the GPU is touched (spawned workers)
    world, rank, local = dist_setup(args)
    dev = torch.device("cuda", local if world > 1 else 0)
    backend = args.backend if world > 1 or args.dist else None
    total_steps = args.envs * world * args.horizon * args.steps
    extra = {}
    if args.learner == "pg":
        wall, phases, mfma, stats = pg_bench(args, world, rank, dev)
        upd = ("1 epoch x 1 minibatch: ratio == 1, an A2C-style step" if args.epochs * args.minibatches == 1
               else f"{args.epochs} epochs x {args.minibatches} minibatches, one Adam step each (PPO extension: "
                    f"time-contiguous minibatch slices, order shuffled per epoch; the reference has no PPO, "
                    f"parity unpinned)")
        if args.sched_restart:
            upd += "; CurriculumScheduler restarted from its initial config every iteration"
        if WORKLOADS[args.config].get("scheduler"):
            upd += f"; success_rule={args.success_rule or 'terminated'}"
        workload = (f"{WORKLOADS[args.config]['desc']} PG iteration: fused actor-MLP(256,256) rollout of "
                    f"{args.horizon} env steps x {args.envs} envs + critic fwd + GAE + adv-norm + PPO-clip / value "
                    f"heads + backward + Adam ({upd})")
        dtype = "bf16 MFMA (f32 acc) + f32/f64 env"
        coll = "RCCL" if backend == "nccl" else "gloo (host-staged)"
        par = (f"dp{world} (env shards; {coll} all-gather of the f64 advantage moments, all-reduce of the f32 "
               f"grads)" if backend else "dp1")
        extra = {"phases_ms": phases, "mfma": mfma, "train_stats": stats}
    else:
        wall, kernel_ms = rollout_bench(args, world, rank, dev)
        workload = (f"config_{args.curriculum}.json fused rollout: run_episode x SimpleLearner, dense reward, "
                    f"{args.horizon} env steps per bench step")
        dtype = "f32+f64"
        par = f"env-shard replicas x{world} (no collective)"
        extra = {"rollout_kernel_ms": round(kernel_ms, 4)}
    value = total_steps / wall
    out = {
        "metric": "env-steps/sec @4096 envs/GPU, 1/2/4/8 MI355X; %HBM roofline step kernel",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic (device Philox4x32-10 reset draws, policy / learner noise; random-init weights)",
        "config": {"workload": workload, "learner": args.learner, "envs_per_gpu": args.envs,
                   "global_envs": args.envs * world, "horizon": args.horizon, "parallelism": par,
                   "world_size": world,
                   "backend": {"nccl": "nccl (RCCL over xGMI)", "gloo": "gloo (harness check, ranks may share a GPU)",
                               None: None}[backend],
                   "ranks_per_gpu": (world + torch.cuda.device_count() - 1) // torch.cuda.device_count()
                   if backend == "gloo" else 1,
                   "overlap_comm": bool(args.overlap), "reserve_cus": args.reserve_cus,
                   "reuse_h2": not args.recompute_h2},
    }
    out.update(extra)
    # peak torch-allocated device memory of the bench itself (trainer buffers, tapes), read
    # before the roofline probe allocates its own
    out["device_memory_gb"] = {"max_allocated": round(torch.cuda.max_memory_allocated(dev) / 1e9, 3),
                               "max_reserved": round(torch.cuda.max_memory_reserved(dev) / 1e9, 3)}
    if rank == 0 and not args.no_roofline:
        out["roofline"] = step_kernel_roofline(args, dev)
        out["step_kernel_at_bench_envs"] = step_kernel_small(args.envs, dev)
    if rank == 0 and cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out))
    if _dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
