"""Vectorised policy-gradient trainer (NEW capability).

The reference's learner is a per-episode random hill-climber
(policies/simple_learner.py); BASELINE.json asks for an MLP(256,256)
actor-critic with GAE and policy gradients on top of the same env.  One
``PGTrainer.iteration()`` =

  1. ``dxrl_pg_rollout``  -- T env steps of every env, actor MLP fused into
     the step kernel (bf16 MFMA), Gaussian sampling, optional fused noise
     injection (robustness_tests.py:140-211), auto-reset, training tape;
  2. critic forward over the T+1 observation blocks (bf16 MFMA GEMMs);
  3. ``dxrl_pg_gae`` reverse scan + advantage normalisation from (count, mean, M2)
     moments merged without cancellation (global across ranks: one all-gather of each
     rank's 3 f64, merged in rank order by ``dxrl_pg_adv_combine``);
  4. actor forward, PPO-clip / value / entropy heads (``dxrl_pg_heads``);
  5. backward GEMMs (input grads with fused tanh' gate, weight grads by
     split-K over samples with the bias as an extra ones-row);
  6. the f32 gradient SUM all-reduce over RCCL (world > 1), in two halves on a side stream:
     the critic's beside the actor's train pass, the actor's before Adam;
  7. global-norm clip + Adam on the f32 master, bf16 repack.

Every matrix contraction runs in libdxrl.so; torch only owns the buffers.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import torch

from . import _native as N
from .distributed import all_gather_into_, all_reduce_sum_, gather_adv_moments_, global_count, loss_scales
from .envs import VecEnv

# csrc/dxrl_pg.h
OBS_IN, IN, H, HX, OUT, ACT, ACT_PAD = 45, 64, 256, 288, 32, 15, 16
H2LD = 264  # row pitch (bf16) of the stored layer-2 activations: the fused learner's H2 tile rows
# rollout kernels (dxrl_pg_rollout_kernel) whose calls write the actor's layer-2 tape
TAPE_KERNELS = (1, 2)
W1, W2, W3 = H * IN, H * HX, OUT * HX
OFF = {"W1a": 0, "W2a": W1, "W3a": W1 + W2, "logstd": W1 + W2 + W3}
OFF["W1c"] = OFF["logstd"] + 32
OFF["W2c"] = OFF["W1c"] + W1
OFF["W3c"] = OFF["W2c"] + W2
NPARAMS = OFF["W3c"] + W3
W2T, W3T = H * H, H * OUT
BF = {"W1a": 0, "W2a": W1, "W3a": W1 + W2, "W2aT": W1 + W2 + W3, "W3aT": W1 + W2 + W3 + W2T}
BF["W1c"] = BF["W3aT"] + W3T
BF["W2c"] = BF["W1c"] + W1
BF["W3c"] = BF["W2c"] + W2
BF["W2cT"] = BF["W3c"] + W3
BF["W3cT"] = BF["W2cT"] + W2T
NBF_ROWS = BF["W3cT"] + W3T  # row-layout copies (GEMM chain, rollout)
# + fragment-ordered streams of W1, W2, W3, W2T, W3T per network (fused learner; dxrl_pg.h kFr*)
NBF = NBF_ROWS + 2 * (H * IN + H * H + OUT * H + H * H + H * OUT)
LOGICAL_PARAMS = 2 * (OBS_IN * H + H) + 2 * (H * H + H) + (H * ACT + ACT) + (H + 1) + ACT  # 159,263


@dataclass
class TrainerConfig:
    """Build-owned knobs (never stored in the reference's strict dataclasses)."""
    horizon: int = 200
    max_steps: Optional[int] = None          # run_episode loop bound; default env.max_episode_steps
    gamma: float = 0.99
    lam: float = 0.95
    clip_eps: float = 0.2
    vf_coef: float = 0.5
    ent_coef: float = 0.0
    lr: float = 3e-4
    betas: tuple = (0.9, 0.999)
    adam_eps: float = 1e-5
    max_grad_norm: float = 0.5
    init_log_std: float = -0.5
    obs_noise_std: float = 0.0               # config C5: 0.05
    dyn_noise_std: float = 0.0               # config C5: 0.05
    seed: int = 0
    splitk_target_blocks: int = 768
    fused: bool = True                       # one-pass learner kernels (dxrl_pg_fused) vs the GEMM chain
    h1_recompute: bool = True                # fused dW2: recompute H1 from obs on chip (no H1 HBM round trip)
    record_cap: int = 0                      # per-env episode records per iteration (0 = off)
    epochs: int = 1                          # PPO epochs over the iteration's samples
    minibatches: int = 1                     # time-contiguous minibatches per epoch, order shuffled per epoch
                                             # (1 x 1: one update, ratio == 1 -- an A2C-style step)
    success_rule: str = "terminated"         # "training" (episode_utils.py:52) or "terminated"
    # collectives on a side stream beside the train passes (True) or on the compute stream between
    # them (False, default): the learner kernels are persistent and fill every CU, so a collective
    # beside them delays them by about its own length and the cross-stream ordering adds the rest;
    # at world 1 over RCCL the overlapped form costs 85 us per iteration, the serialised one 31 us
    # (profiles/r04/ab_dist_overlap.log).  Both give bit-identical results.
    overlap_comm: bool = False
    # CUs left free of the persistent learner kernels (k_pg_fused, k_wgrad_l1): their grids become
    # CUs - reserve_cus, so a collective on the comm stream has CUs of its own to run on beside them
    # (overlap_comm); 0 = every CU.  Changes the learner's per-workgroup partial-sum order (so the
    # gradients' last bits), not the sums themselves; overlapped == serialised holds at any value.
    reserve_cus: int = 0
    # both train passes of a step through dxrl_pg_fused_pair: their dW2 contractions in one launch
    # (learner CUs / 2 splits each instead of every CU per network: half the split-K slab traffic)
    # and both reductions in one launch (needs the fused learner with on-chip H1, serialised
    # exchanges, and more than 16 splits per network after the cap below); False: one
    # dxrl_pg_fused call per network.  Memory: the critic's own dH2 ([M][256] bf16, 0.42 GB at
    # C2's 819,200 samples) and fused-partial slab, and 2 x pair_splits [256][256] f32 dW2 slabs
    # (64 MB at 128 splits); the per-network path's [splits + 16][256][288] slab is then not
    # allocated unless a per-network pass runs
    pair_learner: bool = True
    # dW2 splits per network of the paired step (0: learner CUs / 2), capped at the smallest
    # minibatch slice's 32-row chunk count; the paired step needs the capped count > 16
    pair_splits: int = 0
    # one rank, paired step: the pair's reduction also writes the grad-norm partials
    # (dxrl_pg_fused_pair_gnorm) and the optimiser step finishes the norm from them
    # (dxrl_pg_adam_step) instead of a k_sumsq pass over the gradient -- one launch fewer per
    # update; the norm's f64 sum order differs (agrees to f64 rounding)
    fused_gnorm: bool = True
    # the layer-2 activations of each network computed once per weight version (round 6): the
    # rollout writes the actor's H2 of every sample (16-env rollout kernel), the critic-values pass
    # writes the critic's, and the first train pass under those weights reads them instead of
    # recomputing layer 2 (bit-identical: same MFMA k order and tanh); later PPO passes, after an
    # optimiser step, recompute.  Memory: [M][264] bf16 for the actor (0.43 GB at C2), and as
    # much for the critic when epochs x minibatches == 1 (else its store would cost more than the
    # first minibatch pass saves)
    reuse_h2: bool = True


def minibatch_bounds(M: int, B: int, round_samples: int):
    """Sample offsets of B time-contiguous minibatch slices of M samples.  The fused learner
    runs one 128-sample tile per CU per round (round_samples = 128 x CUs), so a slice of 6.25
    rounds costs 7: slices are cut on whole rounds with the rounds split as evenly as possible
    (4 minibatches of 25 rounds: 7, 6, 6, 6 instead of 4 x 7), the last slice taking the
    remainder.  With fewer rounds than minibatches: equal slices."""
    if B == 1:
        return [0, M]
    R = -(-M // round_samples)
    if R < B:
        size = M // B
        return [k * size for k in range(B)] + [M]
    out = [0]
    for k in range(B):
        out.append(min(M, out[-1] + (R // B + (1 if k < R % B else 0)) * round_samples))
    return out


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class PGTrainer:
    def __init__(self, env: VecEnv, cfg: TrainerConfig = TrainerConfig(), process_group=None, world_size: int = 1):
        if env.reward_type != "dense":
            raise ValueError("the policy-gradient trainer uses the dense reward")
        p_, b_ = C.c_int64(), C.c_int64()
        N.call("dxrl_pg_sizes", C.byref(p_), C.byref(b_))
        assert (p_.value, b_.value) == (NPARAMS, NBF), "csrc/dxrl_pg.h and trainer.py disagree"
        self.env, self.cfg = env, cfg
        self.dev = env.device
        self.n = env.num_envs
        self.T = cfg.horizon
        self.M = self.n * self.T
        if self.M % 32:
            raise ValueError("num_envs * horizon must be a multiple of 32")
        self.max_steps = cfg.max_steps or env.max_episode_steps
        if cfg.epochs < 1 or cfg.minibatches < 1 or self.M % cfg.minibatches or (self.M // cfg.minibatches) % 32:
            raise ValueError("epochs >= 1; num_envs * horizon must split into `minibatches` slices of a multiple "
                             "of 32 samples")
        if (cfg.epochs > 1 or cfg.minibatches > 1) and not cfg.fused:
            raise ValueError("epochs / minibatches need the fused learner")
        self._mb = (0, self.M)  # (first sample, samples) of the minibatch the train passes read
        self._loss_rows = self.M  # rows of the last train pass (loss_stats)
        self.pg = process_group
        self.world = world_size
        # collectives run with several ranks or with an explicit process group (a world-1 group
        # executes the same RCCL calls: bench.py --dist, tests/test_gpu_rccl.py)
        self.collective = process_group is not None or world_size > 1
        # Exchanges that overlap compute (collective mode): the advantage-moment all-gather runs
        # beside the critic's train pass (which does not read the normalisation), the critic
        # half of the gradient all-reduce beside the actor's, the scheduler's code exchange
        # beside critic values.  Element-wise the same SUMs, so results do not change.
        self._comm = None
        if self.collective and cfg.overlap_comm and env.device.type == "cuda":
            self._comm = torch.cuda.Stream(device=env.device)
        self._stats_pending = self._grads_pending = False
        self._stats_event = torch.cuda.Event() if self._comm is not None else None
        self._update_follows = True  # iteration(update=False) clears it for its train passes
        self.global_M = global_count(self.M, self.world, self.pg)  # samples of all ranks per iteration
        if self.global_M != self.M * self.world:
            raise ValueError(f"every rank needs the same num_envs * horizon ({self.M} here, {self.global_M} over "
                             f"{self.world} ranks): the episode-code all-gather and the scheduler's global env ids "
                             "assume equal shards")
        self.step_count = 0
        self.iteration_index = 0
        self.diag_flags = 0  # rollout timing ablations only (see dxrl_pg_rollout_args.diag_flags)
        d, f32, bf, M, n, T = self.dev, torch.float32, torch.bfloat16, self.M, self.n, self.T
        z = lambda *s, dt=f32: torch.zeros(*s, dtype=dt, device=d)  # noqa: E731
        self.params, self.grads, self.m1, self.m2 = z(NPARAMS), z(NPARAMS), z(NPARAMS), z(NPARAMS)
        self._spare = None  # the optimiser's output buffers (params / m1 / m2 ping-pong with these)
        self.packed = z(NBF, dt=bf)
        self._init_params()
        # tape
        self.obs_rm = z((T + 1) * n, IN, dt=bf)
        self.act = z(M, ACT_PAD)
        self.logp, self.rew = z(M), z(M)
        self.done = z(M, dt=torch.uint8)
        self.ep_ret = torch.zeros(n, dtype=torch.float64, device=d)
        self.ep_count = z(n, dt=torch.int32)
        self.ep_sum_ret = torch.zeros(n, dtype=torch.float64, device=d)
        self.ep_sum_len = z(n, dt=torch.int32)
        self.ep_succ = z(n, dt=torch.int32)
        cap = max(0, int(cfg.record_cap))
        self.rec_return = torch.zeros(n, max(cap, 1), dtype=torch.float64, device=d)
        self.rec_length = z(n, max(cap, 1), dt=torch.int32)
        self.rec_success = z(n, max(cap, 1), dt=torch.uint8)
        self.rec_end = z(n, max(cap, 1), dt=torch.int32)
        if cfg.success_rule not in ("training", "terminated"):
            raise ValueError("success_rule must be 'training' or 'terminated'")
        self.scheduler = None
        self.ep_code = None  # u16 [T N] episode-end codes (scheduler feed, attach_curriculum)
        # hidden activations, row-major [rows][288]: columns 0..255 = tanh units, column 256 = 1
        # (the next layer reads K = 256; the weight-gradient GEMM reads I = 288 and gets the bias
        # gradient as column 256)
        # The layer-by-layer GEMM chain (fused=False, the A/B path) stores every activation and
        # head gradient; the fused learner keeps them on chip and needs only dH2 (and H1 in
        # H1-copy mode), so nothing else is allocated for it (C4: ~5 GB less).
        chain = not cfg.fused
        self.H1a = z(M, HX, dt=bf) if chain or not cfg.h1_recompute else None
        self.H2a = self.H1c = self.H2c = self.mu = self.dmu_rm = self.dv_rm = self.dH1 = None
        self.dls_partial = self.loss_partial = None
        if chain:
            self.H2a = z(M, HX, dt=bf)
            self.H1c, self.H2c = z((T + 1) * n, HX, dt=bf), z((T + 1) * n, HX, dt=bf)
            for t in (self.H1a, self.H2a, self.H1c, self.H2c):
                t[:, H].fill_(1.0)
            self.mu = z(M, OUT)
            self.dmu_rm, self.dv_rm = z(M, OUT, dt=bf), z(M, OUT, dt=bf)
            self.dls_partial = z((M + 255) // 256, ACT_PAD)
            self.loss_partial = torch.zeros((M + 255) // 256, 4, dtype=torch.float64, device=d)
            self.dH1 = z(M, H, dt=bf)
        self.V = z(OUT if chain else 1, (T + 1) * n)  # the GEMM chain writes all 32 head rows
        self.adv, self.ret = z(M), z(M)
        self.stats = torch.zeros(8, dtype=torch.float64, device=d)
        self.moments_all = torch.zeros(self.world, 3, dtype=torch.float64, device=d)  # ranks' stats[5..7]
        # shared f64 scratch: the optimiser's 512 grad-norm partials and dxrl_pg_gae's moment triples
        nb = max(512, N.gae_partial_doubles(n, T))
        self.partial = torch.zeros(nb, dtype=torch.float64, device=d)
        self.dH2 = z(M, H, dt=bf)
        cus = int(torch.cuda.get_device_properties(d).multi_processor_count)
        if not 0 <= int(cfg.reserve_cus) < cus:
            raise ValueError(f"reserve_cus must be in [0, {cus})")
        self.learner_cus = cus - int(cfg.reserve_cus)  # CUs the persistent learner grids use
        # dW2: one workgroup per (learner) CU
        self.splits = max(1, min(cfg.splitk_target_blocks // 3, M // 1024))
        if self.learner_cus < cus:
            self.splits = min(self.splits, self.learner_cus)
        self._kpartial = None  # [splits + 16][256][288] f32, allocated on first use (kpartial)
        self.gnorm2 = torch.zeros(1, dtype=torch.float64, device=d)
        tr_, pf_ = C.c_int32(), C.c_int64()
        N.call("dxrl_pg_fused_sizes", C.byref(tr_), C.byref(pf_))
        # up to two learner workgroups per CU (64-sample tiles); the library clamps to its geometry
        # (one 128-sample workgroup per CU), so a reservation passes the CU count itself
        self.fused_grid = 2 * cus if self.learner_cus == cus else self.learner_cus
        self.fused_partial = z(self.fused_grid + 17, pf_.value)  # + reduction scratch and sum
        self.fused_loss = torch.zeros(self.fused_grid, 4, dtype=torch.float64, device=d)
        # paired learner step (dxrl_pg_fused_pair): the critic's own dH2 / partial buffers, the
        # per-network dW2 split count (every minibatch slice must give each split > 16 chunks)
        mb_rows = min(b - a for a, b in zip(self.minibatch_bounds()[:-1], self.minibatch_bounds()[1:]))
        if int(cfg.pair_splits) < 0:
            raise ValueError("pair_splits must be >= 0 (0: learner CUs / 2)")
        self.pair_splits = min(int(cfg.pair_splits) or self.learner_cus // 2, mb_rows // 32)
        self.paired = (cfg.pair_learner and cfg.fused and cfg.h1_recompute and self._comm is None
                       and self.pair_splits > 16 and all(x % 32 == 0 for x in self.minibatch_bounds()))
        self.dH2c = self.fused_partial_c = self.kpartial_c = self.kpartial_a = None
        if self.paired:
            self.dH2c = z(M, H, dt=bf)
            self.fused_partial_c = z(self.fused_grid + 17, pf_.value)
            self.kpartial_a = z(self.pair_splits, H, H)
            self.kpartial_c = z(self.pair_splits, H, H)
        # grad-norm partials of the last paired step's reduction (one rank only: sharded, the
        # all-reduce changes the gradient after them); _gn_blocks > 0 while they match the grads
        self.gn_partial, self._gn_blocks = None, 0
        if self.paired and cfg.fused_gnorm and not self.collective:
            nbk = C.c_int32()
            N.call("dxrl_pg_gnorm_blocks", C.byref(nbk))
            self.gn_partial = torch.zeros(nbk.value, dtype=torch.float64, device=d)
        # layer-2 activations for the first train pass of a weight version (cfg.reuse_h2)
        self.h2a = self.h2c = None
        self._h2a_fresh = self._h2c_fresh = self.h2a_tape_written = False
        if cfg.fused and cfg.reuse_h2:
            # the actor's tape is allocated by the first rollout that runs the 16-env kernel (the
            # only one that writes it: not at C4's 8192 envs, where it would be 0.86 GB unused)
            # the critic's only when one full-batch train pass reads it: the values pass pays the
            # store (≈40 µs at C2) on every iteration, a PPO minibatch pass saves a quarter of it
            if cfg.epochs * cfg.minibatches == 1:
                self.h2c = z(M + n, H2LD, dt=bf)
        self.pack()

    @property
    def kpartial(self):
        """Split-K partial slabs of the per-network dW2 paths (+ two-level reduction scratch):
        allocated on first use, so a paired-step trainer that never runs a per-network pass does
        not hold them."""
        if self._kpartial is None:
            self._kpartial = torch.zeros(self.splits + 16, H, HX, dtype=torch.float32, device=self.dev)
        return self._kpartial

    @kpartial.setter
    def kpartial(self, t):
        self._kpartial = t

    # ------------------------------------------------------------------ params
    def _view(self, t, off, rows, cols):
        return t[off:off + rows * cols].view(rows, cols)

    def block(self, name, t=None):
        t = self.params if t is None else t
        shape = {"W1": (H, IN), "W2": (H, HX), "W3": (OUT, HX)}[name[:2]]
        return self._view(t, OFF[name], *shape)

    def _init_params(self):
        g = torch.Generator(device="cpu").manual_seed(int(self.cfg.seed))
        for net, head_rows, head_gain in (("a", ACT, 0.01), ("c", 1, 1.0)):
            for name, rows, cols, gain in ((f"W1{net}", H, OBS_IN, math.sqrt(2)), (f"W2{net}", H, H, math.sqrt(2)),
                                           (f"W3{net}", head_rows, H, head_gain)):
                w = torch.empty(rows, cols)
                torch.nn.init.orthogonal_(w, gain=gain, generator=g)
                self.block(name)[:rows, :cols].copy_(w.to(self.dev))
        self.params[OFF["logstd"]:OFF["logstd"] + ACT].fill_(self.cfg.init_log_std)

    def pack(self):
        N.call("dxrl_pg_pack_weights", self.dev.index, N.ptr(self.params), N.ptr(self.packed), self._s())
        self._h2a_fresh = self._h2c_fresh = False  # new weights: the stored activations are stale

    def _s(self):
        return N.stream_of(self.dev)

    def _bf(self, name):
        return self.packed[BF[name]:]

    # ------------------------------------------------------------------ launches
    def _gemm(self, A, lda, Bt, ldb, M, Nn, K, *, bias=None, bias_stride=0, act=0, gate=None, ldg=0, Cf=None,
              ldcf=0, Crm=None, ldc=0, Cfm=None, ldfm=0, Cffm=None, ldffm=0, splits=1, partial=None):
        p = N.ptr
        N.call("dxrl_gemm_bf16", self.dev.index, p(A), lda, p(Bt), ldb, M, Nn, K, p(bias), bias_stride, act, p(gate),
               ldg, p(Cf), ldcf, p(Crm), ldc, p(Cfm), ldfm, p(Cffm), ldffm, splits, p(partial), self._s())

    def _wgrad(self, Y, ldy, O, X, ldx, I, dst):
        """dst[O][I] = sum_m Y[m][:O] X[m][:I] (row-major operands, split-K over samples)."""
        p = N.ptr
        N.call("dxrl_wgrad_bf16", self.dev.index, p(Y), ldy, O, p(X), ldx, I, self.M, self.splits,
               p(self.kpartial), p(dst), self._s())

    def rollout(self):
        a = N.PgRolloutArgs()
        a.horizon, a.max_steps = self.T, self.max_steps
        a.policy_seed = (int(self.cfg.seed) * 0x9E3779B97F4A7C15 + 17) & (2**64 - 1)
        a.iteration = self.iteration_index
        a.obs_noise_std, a.dyn_noise_std = self.cfg.obs_noise_std, self.cfg.dyn_noise_std
        p = N.ptr
        a.obs_rm, a.obs_fm, a.act, a.logp, a.rew, a.done = (p(self.obs_rm), None, p(self.act), p(self.logp),
                                                            p(self.rew), p(self.done))
        a.ep_return, a.ep_count, a.ep_sum_return = p(self.ep_ret), p(self.ep_count), p(self.ep_sum_ret)
        a.ep_sum_length, a.ep_successes = p(self.ep_sum_len), p(self.ep_succ)
        a.diag_flags = self.diag_flags
        a.success_rule = N.SUCCESS_TERMINATED if self.cfg.success_rule == "terminated" else N.SUCCESS_TRAINING
        a.record_cap = max(0, int(self.cfg.record_cap))
        a.rec_return, a.rec_length = p(self.rec_return), p(self.rec_length)
        a.rec_success, a.rec_end_step = p(self.rec_success), p(self.rec_end)
        a.ep_code = p(self.ep_code)
        a.applied_act = p(getattr(self, "applied_act", None))  # parity tapes (tests only; None in runs)
        a.dyn_noise_tape = p(getattr(self, "dyn_noise_tape", None))
        a.obs_noise_tape = p(getattr(self, "obs_noise_tape", None))
        # the actor's H2 tape (written by the 16- and 32-env kernels, not the 64-env reference one)
        tape = False
        if self.cfg.fused and self.cfg.reuse_h2:
            k = C.c_int32()
            N.call("dxrl_pg_rollout_kernel", self.env.handle, self.diag_flags, C.byref(k))
            tape = k.value in TAPE_KERNELS
            if tape and self.h2a is None:  # zero padding columns (the learner's LDS-DMA reads them)
                self.h2a = torch.zeros(self.M, H2LD, dtype=torch.bfloat16, device=self.dev)
        a.h2_tape = p(self.h2a) if tape else None
        N.call("dxrl_pg_rollout", self.env.handle, p(self.packed), p(self.params), C.byref(a), self._s())
        self._h2a_fresh = self.h2a_tape_written = tape

    def _mlp_forward(self, net, rows, H1, H2, head_f32=None, head_fm=None, ld_head_fm=0):
        P = self.params
        self._gemm(self.obs_rm, IN, self._bf(f"W1{net}"), IN, rows, H, IN, act=1, Crm=H1, ldc=HX)  # bias = col 45
        self._gemm(H1, HX, self._bf(f"W2{net}"), HX, rows, H, H, bias=P[OFF[f"W2{net}"] + H:], bias_stride=HX, act=1,
                   Crm=H2, ldc=HX)
        self._gemm(H2, HX, self._bf(f"W3{net}"), HX, rows, OUT, H, bias=P[OFF[f"W3{net}"] + H:], bias_stride=HX,
                   Cf=head_f32, ldcf=OUT, Cffm=head_fm, ldffm=ld_head_fm)

    def critic_forward(self):
        rows = self.M + self.n  # T + 1 observation blocks (bootstrap values)
        self._mlp_forward("c", rows, self.H1c, self.H2c, head_fm=self.V, ld_head_fm=rows)

    def actor_forward(self):
        self._mlp_forward("a", self.M, self.H1a, self.H2a, head_f32=self.mu)

    # ------------------------------------------------------------------ fused path
    def _fused_args(self, net, train, rows, start=0):
        c, p = self.cfg, N.ptr
        f = N.PgFusedArgs()
        f.net, f.train, f.rows = net, int(train), rows
        f.packed, f.params, f.obs = p(self.packed), p(self.params), p(self.obs_rm[start:])
        f.act, f.logp_old, f.adv, f.ret = p(self.act[start:]), p(self.logp[start:]), p(self.adv[start:]), \
            p(self.ret[start:])
        f.stats = p(self.stats)
        # each pass is one gradient step on the mean loss over its samples of all ranks (equal
        # shards: rows per rank x world)
        f.inv_total_samples, f.ent_coef = loss_scales(rows * self.world, self.world, c.ent_coef)
        f.clip_eps, f.vf_coef = c.clip_eps, c.vf_coef
        f.values = p(self.V[0])
        f.h1, f.dh2 = p(self.H1a), p(self.dH2)
        f.partial, f.loss_partial, f.grid = p(self.fused_partial), p(self.fused_loss), self.fused_grid
        f.wgrad_splits, f.wgrad_partial, f.grads = self.splits, p(self.kpartial), p(self.grads)
        f.h1_mode = 0 if c.h1_recompute else 1
        if train and (self._h2c_fresh if net == 1 else self._h2a_fresh):
            f.h2_in = p((self.h2c if net == 1 else self.h2a)[start:])
        return f

    def train(self):
        """Both train passes of the step (critic, then actor) with their dW2 contractions in one
        launch and both networks' reductions in one launch (dxrl_pg_fused_pair)."""
        start, rows = self._mb
        self._loss_rows = rows
        if self._stats_pending:
            torch.cuda.current_stream(self.dev).wait_event(self._stats_event)
            self._stats_pending = False
        fc, fa = self._fused_args(1, True, rows, start), self._fused_args(0, True, rows, start)
        p = N.ptr
        fc.dh2, fc.partial, fc.wgrad_partial = p(self.dH2c), p(self.fused_partial_c), p(self.kpartial_c)
        fa.wgrad_partial = p(self.kpartial_a)
        fc.wgrad_splits = fa.wgrad_splits = self.pair_splits
        if self.gn_partial is not None:
            nb = C.c_int32()
            N.call("dxrl_pg_fused_pair_gnorm", self.dev.index, C.byref(fc), C.byref(fa), p(self.gn_partial),
                   self.gn_partial.numel(), C.byref(nb), self._s())
            self._gn_blocks = nb.value
        else:
            N.call("dxrl_pg_fused_pair", self.dev.index, C.byref(fc), C.byref(fa), self._s())

    def critic_values(self):
        """V over the T + 1 observation blocks (fused forward, nothing stored but V)."""
        f = self._fused_args(1, False, self.M + self.n)
        f.h2_out = N.ptr(self.h2c)  # (None: not stored)
        N.call("dxrl_pg_fused", self.dev.index, C.byref(f), self._s())
        self._h2c_fresh = self.h2c is not None

    def actor_train(self):
        start, rows = self._mb
        self._loss_rows = rows
        self._gn_blocks = 0  # this pass rewrites the gradient: the pair's norm partials are stale
        if self._stats_pending:  # the actor's head normalises the advantages with the global moments
            # only the moments: the critic half's all-reduce queued behind them on the comm stream
            # runs beside this pass
            torch.cuda.current_stream(self.dev).wait_event(self._stats_event)
            self._stats_pending = False
        N.call("dxrl_pg_fused", self.dev.index, C.byref(self._fused_args(0, True, rows, start)), self._s())

    def critic_train(self):
        start, rows = self._mb
        self._loss_rows = rows
        self._gn_blocks = 0
        N.call("dxrl_pg_fused", self.dev.index, C.byref(self._fused_args(1, True, rows, start)), self._s())
        # the critic half's SUM all-reduce runs beside the actor's pass -- only when an optimiser
        # step follows (iteration(update=False) issues no gradient collective, as the serialised
        # form does not, and leaves nothing in flight that the next pass's gradients would race)
        if self._comm is not None and self._update_follows:
            with self._on_comm():
                self._allreduce(self.grads[OFF["W1c"]:])
            self._grads_pending = True

    def ppo_updates(self):
        """epochs x minibatches PPO-clip updates (actor + critic pass and an Adam step each)
        over time-contiguous slices of the iteration's samples; the slice order is a fresh
        permutation per epoch (seeded by cfg.seed and the iteration)."""
        c = self.cfg
        bounds = self.minibatch_bounds()
        rng = np.random.default_rng([int(c.seed), self.iteration_index])
        for _ in range(c.epochs):
            for k in rng.permutation(c.minibatches):
                self._mb = (bounds[k], bounds[k + 1] - bounds[k])
                self.train_passes()
                self.optimizer_step()
        self._mb = (0, self.M)

    def train_passes(self):
        """The step's two train passes: paired (train) or one call per network."""
        if self.paired:
            self.train()
        else:
            self.critic_train()
            self.actor_train()

    def minibatch_bounds(self):
        return minibatch_bounds(self.M, self.cfg.minibatches, 128 * self.learner_cus)

    def phases(self):
        """The iteration's launch groups in order (bench.py times each)."""
        if self.cfg.fused and self.cfg.epochs * self.cfg.minibatches > 1:
            ph = ["rollout", "critic_values", "advantages", "ppo_updates"]
        elif self.cfg.fused and self.paired:
            ph = ["rollout", "critic_values", "advantages", "train", "optimizer_step"]
        elif self.cfg.fused:
            # the critic first: its pass does not need the (all-gathered) normalisation moments
            ph = ["rollout", "critic_values", "advantages", "critic_train", "actor_train", "optimizer_step"]
        else:
            ph = ["rollout", "critic_forward", "advantages", "actor_forward", "heads", "backward", "optimizer_step"]
        if self.scheduler is not None:  # feed launched behind the rollout, applied after the learner
            ph = ph[:1] + ["schedule_feed"] + ph[1:] + ["schedule_apply"]
        return ph

    def _allreduce(self, t):
        all_reduce_sum_(t, self.world, self.pg)

    def advantages(self):
        c = self.cfg
        N.call("dxrl_pg_gae", self.dev.index, N.ptr(self.rew), N.ptr(self.done), N.ptr(self.V[0]), self.n, self.T,
               c.gamma, c.lam, N.ptr(self.adv), N.ptr(self.ret), N.ptr(self.partial), N.ptr(self.stats), self._s())
        # every rank's (count, mean, M2) in rank order, merged on device (identical on all ranks);
        # one rank: dxrl_pg_gae already wrote the combined statistics
        if self.collective:
            with self._on_comm():
                gather_adv_moments_(self.moments_all, self.stats, self.world, self.pg)
                N.call("dxrl_pg_adv_combine", self.dev.index, N.ptr(self.moments_all), self.world,
                       N.ptr(self.stats), self._s())
                if self._comm is not None:
                    self._stats_event.record(self._comm)
            self._stats_pending = self._comm is not None

    def _on_comm(self):
        """Context for an exchange: the comm stream (after everything enqueued so far on the
        compute stream), or the compute stream itself without overlap."""
        if self._comm is None:
            return _null()
        self._comm.wait_stream(torch.cuda.current_stream(self.dev))
        return torch.cuda.stream(self._comm)

    def _join_comm(self):
        """The compute stream waits for every exchange issued so far."""
        if self._comm is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self._comm)
        self._stats_pending = self._grads_pending = False

    def heads(self):
        c, p = self.cfg, N.ptr
        h = N.PgHeadsArgs()
        h.mu, h.values, h.act, h.logp_old = p(self.mu), p(self.V[0]), p(self.act), p(self.logp)
        h.adv, h.ret, h.stats, h.params = p(self.adv), p(self.ret), p(self.stats), p(self.params)
        h.num_samples = self.M
        h.inv_total_samples, h.ent_coef = loss_scales(self.global_M, self.world, c.ent_coef)
        h.clip_eps, h.vf_coef = c.clip_eps, c.vf_coef
        h.dmu_rm, h.dmu_fm, h.dv_rm, h.dv_fm = p(self.dmu_rm), None, p(self.dv_rm), None
        h.dlogstd_partial, h.loss_partial, h.grads = p(self.dls_partial), p(self.loss_partial), p(self.grads)
        N.call("dxrl_pg_heads", self.dev.index, C.byref(h), self._s())

    def backward(self):
        M, G = self.M, self.grads
        for net, dY, H1, H2 in (("a", self.dmu_rm, self.H1a, self.H2a), ("c", self.dv_rm, self.H1c, self.H2c)):
            self._wgrad(dY, OUT, OUT, H2, HX, HX, self.block(f"W3{net}", G))
            self._gemm(dY, OUT, self._bf(f"W3{net}T"), OUT, M, H, OUT, gate=H2, ldg=HX, Crm=self.dH2, ldc=H)
            self._wgrad(self.dH2, H, H, H1, HX, HX, self.block(f"W2{net}", G))
            self._gemm(self.dH2, H, self._bf(f"W2{net}T"), H, M, H, H, gate=H1, ldg=HX, Crm=self.dH1, ldc=H)
            self._wgrad(self.dH1, H, H, self.obs_rm, IN, IN, self.block(f"W1{net}", G))

    def optimizer_step(self):
        """Gradient all-reduce (collective mode), then dxrl_pg_optimizer_step: grad-norm partials
        + one clipped-Adam-and-pack launch writing the next master / moments into the spare
        buffers, which then become current (params / m1 / m2 are swapped, not copied)."""
        c = self.cfg
        if self._grads_pending:  # critic half already in flight on the comm stream
            self._allreduce(self.grads[:OFF["W1c"]])
            self._join_comm()
        else:
            self._allreduce(self.grads)
        self.step_count += 1
        if self._spare is None:
            self._spare = tuple(torch.empty_like(t) for t in (self.params, self.m1, self.m2))
        po, m1o, m2o = self._spare
        if self._gn_blocks:  # one rank: the paired reduction left the norm's partials (no k_sumsq)
            N.call("dxrl_pg_adam_step", self.dev.index, N.ptr(self.params), N.ptr(self.grads), N.ptr(self.m1),
                   N.ptr(self.m2), N.ptr(po), N.ptr(m1o), N.ptr(m2o), NPARAMS, c.lr, c.betas[0], c.betas[1],
                   c.adam_eps, self.step_count, c.max_grad_norm, N.ptr(self.gn_partial), self._gn_blocks,
                   N.ptr(self.gnorm2), N.ptr(self.packed), self._s())
            self._gn_blocks = 0
        else:
            N.call("dxrl_pg_optimizer_step", self.dev.index, N.ptr(self.params), N.ptr(self.grads), N.ptr(self.m1),
                   N.ptr(self.m2), N.ptr(po), N.ptr(m1o), N.ptr(m2o), NPARAMS, c.lr, c.betas[0], c.betas[1],
                   c.adam_eps, self.step_count, c.max_grad_norm, N.ptr(self.partial), N.ptr(self.gnorm2),
                   N.ptr(self.packed), self._s())
        self._spare = (self.params, self.m1, self.m2)
        self.params, self.m1, self.m2 = po, m1o, m2o
        self._h2a_fresh = self._h2c_fresh = False  # new weights: the stored activations are stale

    def attach_curriculum(self, scheduler):
        """Host-side CurriculumScheduler (experiments/curriculum_scheduler.py) fed with every
        episode the iteration finished, on all ranks, in (end step, global env id) order -- the
        order evaluation/component_ablation.py:160-170 feeds one process's episodes in.  A
        progression pushes the new config into the device table (effective at each env's next
        reset, as component_ablation.py:165-166 swaps it between episodes).

        The rollout writes one u16 episode-end code per (step, env) and dxrl_sched_scan walks
        them on the device.  With history="window" and the base success-window rule only a few
        numbers cross PCIe (apply_device_summary); sharded, the ranks exchange compact packs
        instead of their codes (dxrl_sched_pack: per-step sums, the rank's last `window` codes,
        and one success bit per episode only while progressions remain;
        dxrl_sched_scan_packed + one all-reduce of <= 64 candidate step counts).  Otherwise
        (history="full", StepBasedScheduler, > 64 pending progressions) every rank's codes are
        all-gathered, copied to the host and fed through update_batch.  Either way every rank's
        scheduler sees the same global stream, so all ranks progress together."""
        self.scheduler = scheduler
        self.env.set_curriculum(scheduler.get_current_config())
        d, n, T = self.dev, self.n, self.T
        self.ep_code = torch.zeros(T * n, dtype=torch.int16, device=d)
        self.codes_all = self.ep_code if not self.collective else None  # host mode's all-gather (lazy)
        w = max(1, int(scheduler.window_size))
        self._sched_w = w
        # one staging block each way, so a feed is one H2D and one D2H copy (each small copy is a
        # ~5 us blit on the stream): in = [tail_len i32][tail i16 x w]; out = [summary i64 x S]
        # [tail_len i32][tail i16 x w]
        S = 4 + 3 * N.SCHED_MAX_CANDIDATES
        self._sched_in_host = torch.zeros(4 + 2 * w, dtype=torch.uint8).pin_memory()
        self._sched_in_dev = torch.zeros(4 + 2 * w, dtype=torch.uint8, device=d)
        self._sched_out_dev = torch.zeros(8 * S + 4 + 2 * w, dtype=torch.uint8, device=d)
        self._sched_out_host = torch.zeros(8 * S + 4 + 2 * w, dtype=torch.uint8).pin_memory()
        self._tail_len_host = self._sched_in_host[:4].view(torch.int32)
        self._tail_in_host = self._sched_in_host[4:].view(torch.int16)
        self._tail_len_in_dev = self._sched_in_dev[:4].view(torch.int32)
        self._tail_in_dev = self._sched_in_dev[4:].view(torch.int16)
        self._summary = self._sched_out_dev[:8 * S].view(torch.int64)
        self._tail_len_out_dev = self._sched_out_dev[8 * S:8 * S + 4].view(torch.int32)
        self._tail_out_dev = self._sched_out_dev[8 * S + 4:].view(torch.int16)
        self._summary_host = self._sched_out_host[:8 * S].view(torch.int64)
        self._tail_out_host = self._sched_out_host[8 * S + 4:].view(torch.int16)
        nb = C.c_int64()
        # sharded: the packed exchange (dxrl_sched_pack holds a step's episode steps in u32)
        self._packed = self.collective and n < (1 << 18)
        if self._packed:
            import torch.distributed as dist
            self.rank = dist.get_rank(self.pg) if self.pg is not None else dist.get_rank()
            wb = C.c_int64()
            N.call("dxrl_sched_pack_words", T, n, w, 1, C.byref(wb))
            self._pack = torch.zeros(wb.value, dtype=torch.int32, device=d)
            self._packs_all = torch.zeros(self.world * wb.value, dtype=torch.int32, device=d)
            self._where = torch.zeros(N.SCHED_MAX_CANDIDATES, 3, dtype=torch.int32, device=d)
            self._cand_steps = torch.zeros(N.SCHED_MAX_CANDIDATES, dtype=torch.int64, device=d)
            N.call("dxrl_sched_packed_scratch_bytes", self.world, T, n, w, C.byref(nb))
        else:
            N.call("dxrl_sched_scratch_bytes", 1, T, n, w, C.byref(nb))
        self._sched_scratch = torch.empty(nb.value, dtype=torch.uint8, device=d)
        self._codes_host = None
        self._sched_event = torch.cuda.Event()
        self._sched_mode = None

    def schedule_feed(self):
        """Behind the rollout: all-gather the episode-end codes, scan them on the device and
        start the (tiny) summary copy; schedule_apply() consumes it after the learner."""
        with self._on_comm():  # beside critic values (collective mode)
            self._schedule_feed()

    def _schedule_feed(self):
        sc = self.scheduler
        P = sc.remaining_progressions(N.SCHED_MAX_CANDIDATES)
        device = sc.history == "window" and sc._uses_success_window_rule() and P <= N.SCHED_MAX_CANDIDATES
        if device and self.collective and not self._packed:
            device = False  # the full-codes exchange below (very large shards)
        if device:
            w = self._sched_w
            # the host lists are authoritative for the window carried in (success bits are all
            # the scan reads); pinned staging, so the copies queue behind the rollout without a
            # host sync (the previous iteration's copies finished before its schedule_apply)
            tail = sc.episode_successes[-w:]
            self._tail_len_host[0] = len(tail)
            if tail:
                self._tail_in_host[:len(tail)] = torch.tensor(tail, dtype=torch.int16)
            self._sched_in_dev.copy_(self._sched_in_host, non_blocking=True)
            a = N.SchedPackedArgs() if self.collective else N.SchedArgs()
            a.window, a.max_candidates, a.threshold = w, P, float(sc.success_rate_threshold)
            a.min_episodes, a.episodes_before = int(sc.min_episodes_before_progression), int(sc.total_episodes)
            a.tail_in, a.tail_len_in = N.ptr(self._tail_in_dev), N.ptr(self._tail_len_in_dev)
            a.tail_out, a.tail_len_out = N.ptr(self._tail_out_dev), N.ptr(self._tail_len_out_dev)
            a.scratch, a.scratch_bytes, a.summary = N.ptr(self._sched_scratch), self._sched_scratch.numel(), \
                N.ptr(self._summary)
            a.world, a.horizon, a.num_envs = self.world, self.T, self.n
            if not self.collective:  # one rank, no exchange: scan the codes themselves
                a.codes = N.ptr(self.ep_code)
                N.call("dxrl_sched_scan", self.dev.index, C.byref(a), self._s())
            else:
                self._packed_feed(a, P)
            self._sched_out_host.copy_(self._sched_out_dev, non_blocking=True)
            self._sched_mode = "device"
        else:
            if self.codes_all is None:
                self.codes_all = torch.zeros(self.world * self.T * self.n, dtype=torch.int16, device=self.dev)
            all_gather_into_(self.codes_all, self.ep_code, self.world, self.pg)
            if self._codes_host is None:
                self._codes_host = torch.zeros(self.codes_all.numel(), dtype=torch.int16).pin_memory()
            self._codes_host.copy_(self.codes_all, non_blocking=True)
            self._sched_mode = "host"
        self._sched_event.record(torch.cuda.current_stream(self.dev))  # the comm stream in collective mode

    def _packed_feed(self, a, P):
        """Sharded device feed: pack -> all-gather the packs -> scan them -> (candidates) the
        owners' in-block step counts, SUM over ranks -> finished summary.  The success bits
        travel only while progressions are still possible (P > 0)."""
        bits = 1 if P > 0 else 0
        wd = C.c_int64()
        N.call("dxrl_sched_pack_words", self.T, self.n, self._sched_w, bits, C.byref(wd))
        W = wd.value
        pack, packs = self._pack[:W], self._packs_all[:self.world * W]
        s = self._s()
        N.call("dxrl_sched_pack", self.dev.index, N.ptr(self.ep_code), self.T, self.n, self._sched_w, bits,
               N.ptr(pack), s)
        all_gather_into_(packs, pack, self.world, self.pg)
        a.packs, a.pack_words, a.bits, a.where = N.ptr(packs), W, bits, N.ptr(self._where)
        N.call("dxrl_sched_scan_packed", self.dev.index, C.byref(a), s)
        if P > 0:
            N.call("dxrl_sched_candidate_steps", self.dev.index, N.ptr(self.ep_code), self.T, self.n, self.rank, P,
                   N.ptr(self._where), N.ptr(self._summary), N.ptr(self._cand_steps), s)
            all_reduce_sum_(self._cand_steps[:P], self.world, self.pg)
            N.call("dxrl_sched_finish", self.dev.index, N.ptr(self._cand_steps), N.ptr(self._summary), s)

    def schedule_apply(self):
        """Replay the iteration's episodes into the scheduler; push a progression to the env."""
        sc = self.scheduler
        self._sched_event.synchronize()
        if self._sched_mode == "device":
            s = self._summary_host.numpy()
            E, S, U, found = (int(x) for x in s[:4])
            cands = s[4:4 + 3 * found].reshape(found, 3)
            w = self._sched_w
            nl = min(w, len(sc.episode_successes[-w:]) + E)
            tail = self._tail_out_host.numpy().view(np.uint16)[:nl][nl - min(w, E):]
            progressed = sc.apply_device_summary(E, S, U, cands, tail)
        else:
            codes = self._codes_host.numpy().view(np.uint16).reshape(self.world, self.T, self.n)
            ep = codes.transpose(1, 0, 2).ravel()
            ep = ep[ep != 0].astype(np.int64)
            progressed = sc.update_batch((ep & 1).astype(bool), ep >> 1)
        if progressed:  # enqueued behind the learner, no host sync (effective at each env's next reset)
            self.env.set_curriculum_async(sc.get_current_config())

    def episode_records(self):
        from .training import gather_records
        rec = gather_records(self.ep_count, self.cfg.record_cap, self.rec_return, self.rec_length,
                             self.rec_success, self.rec_end, self.env._cfg.global_env_offset)
        if rec.dropped:
            import warnings
            warnings.warn(f"{rec.dropped} finished episodes did not fit TrainerConfig.record_cap="
                          f"{self.cfg.record_cap} records per env (an env can finish up to horizon="
                          f"{self.T} episodes per iteration)", RuntimeWarning, stacklevel=2)
        return rec

    def iteration(self, update: bool = True):
        from . import profiling
        marks = profiling.enabled()
        self._update_follows = update
        try:
            for name in self.phases():
                with profiling.range_(f"pg.{name}") if marks else _null():
                    if name == "ppo_updates" and not update:
                        self.train_passes()
                    elif name != "optimizer_step" or update:
                        getattr(self, name)()
        finally:
            self._update_follows = True
        if not update:
            self._join_comm()  # nothing of this iteration's exchanges stays in flight
        self.iteration_index += 1

    # ------------------------------------------------------------------ stats
    def episode_stats(self) -> Dict[str, float]:
        cnt = int(self.ep_count.sum().item())
        out = {"episodes": cnt, "env_steps": self.M}
        if cnt:
            out["mean_return"] = float(self.ep_sum_ret.sum().item()) / cnt
            out["mean_length"] = float(self.ep_sum_len.sum().item()) / cnt
            out["success_rate"] = float(self.ep_succ.sum().item()) / cnt
        return out

    def loss_stats(self) -> Dict[str, float]:
        """Loss terms of the last train pass (the last minibatch of the last epoch), per sample of
        that pass (the fused kernel zeroes the loss rows of workgroups a pass did not launch)."""
        rows = self._loss_rows if self.cfg.fused else self.M
        s = (self.fused_loss if self.cfg.fused else self.loss_partial).sum(0).cpu().numpy() / rows
        return {"policy_loss": float(s[0]), "value_mse": float(s[1]), "clip_frac": float(s[2]),
                "approx_kl": float(s[3]), "grad_norm": float(np.sqrt(self.gnorm2.item()))}
