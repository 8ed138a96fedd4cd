"""Evaluation drivers on the device episode-program kernel (``dxrl_evaluate``).

Drop-ins for
  evaluation/evaluator.py:17-271         ``Evaluator`` (held-out objects, frozen policy)
  evaluation/robustness_tests.py:212-407 ``RobustnessTester`` (noise sweeps)
with the reference's constructor arguments, method names and result dicts.

Every episode runs inside ``k_eval`` (csrc/dxrl_eval.hip); the host only
resolves random streams and assembles result dicts.  Two execution forms:

* ``parallel=False`` (default) -- the reference's exact order.  The reference
  policies draw from ONE process-global stream (np.random for SimpleLearner /
  HeuristicPolicy, the action space's generator for RandomPolicy), consumed
  serially across every episode of the driver loop, and RobustnessTester keeps
  the object where the previous episode left it (manipulation_env.py:156-161).
  Both make episode k depend on episode k-1, so the driver loop runs as ONE
  device lane whose segments are the loop's env instances.  Results equal the
  reference's bit for bit (tests/golden/eval_golden.json) and the host stream
  is left exactly where the reference would leave it.
* ``parallel=True`` -- one lane per episode, each a fresh env instance with its
  own policy stream: either replayed from ``policy_seeds`` (the reference with
  ``np.random.seed(s)`` before each episode -- bit-exact, golden-tested) or, by
  default, device Philox streams keyed by (device_seed, lane) with device reset
  draws (throughput form; distributionally equivalent, not the reference's
  numbers).

The kernel compiles the reference's three policies (all obs-independent): a
frozen SimpleLearner (its ``mean_action`` + exploration noise), HeuristicPolicy
and RandomPolicy.  Any other object with ``select_action`` runs the same plan
through the Gymnasium facade (device env steps, host policy calls, the
reference's loop as written).  With a ``failure_logger``
(failures.FailureLogger) the kernel also records observation / action
trajectories and every failed episode is logged as evaluator.py:101-179 does.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from .envs import ACTION_DIM, RESET_SLOTS, VecEnv, resolve_reset_draws
from .metrics import EvaluationMetrics, HistoryMoments, aggregate_columns, classify_columns, failure_names

OBS_DIM = 45
_MAX_TAPE = 1 << 26  # f64 draws per host tape (512 MB); beyond it use parallel=True


def _pcg(seed):
    return np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))


# ------------------------------------------------------------------ policy streams
class _HostStream:
    """A host random stream the device consumes through a tape: ``draw(n)``
    peeks n raw values without advancing, ``commit(k)`` advances by k."""

    def __init__(self, peek, advance):
        self._peek, self._advance = peek, advance

    def draw(self, n: int) -> np.ndarray:
        return self._peek(n)

    def commit(self, k: int):
        if k:
            self._advance(k)


def _legacy_global(method: str) -> _HostStream:
    """np.random's global RandomState: 'standard_normal' (np.random.normal(0, s) =
    0 + s * gauss, simple_learner.py:60) or 'random_sample' (np.random.uniform,
    heuristic_policy.py:58)."""

    def peek(n):
        st = np.random.get_state()
        v = getattr(np.random, method)(n)
        np.random.set_state(st)
        return v

    return _HostStream(peek, lambda k: getattr(np.random, method)(k))


def _generator_doubles(gen: np.random.Generator) -> _HostStream:
    """Generator.uniform(low, high) consumes one next_double per element (Box.sample)."""

    def peek(n):
        st = gen.bit_generator.state
        v = gen.random(n)
        gen.bit_generator.state = st
        return v

    return _HostStream(peek, lambda k: gen.random(k))


@dataclass
class _PolicyProgram:
    kind: int
    mean: Optional[np.ndarray]
    sigma: float
    stream: _HostStream
    seeded: Any  # seed -> fresh per-episode stream tape of n values


def compiled_program(policy) -> Optional[_PolicyProgram]:
    """policy_program, or None for a policy the kernel does not compile (host-policy path)."""
    try:
        return policy_program(policy)
    except TypeError:
        return None


def policy_program(policy) -> _PolicyProgram:
    """Map a reference policy object onto a DXRL_EVAL_POLICY_* program."""
    name = type(policy).__name__
    space = getattr(policy, "action_space", None)
    if space is not None:
        low, high = np.asarray(space.low), np.asarray(space.high)
        if low.shape != (ACTION_DIM,) or not (np.all(low == -1.0) and np.all(high == 1.0)):
            raise ValueError("the evaluation kernel compiles the reference's Box(-1, 1, (15,)) action space")
    if hasattr(policy, "mean_action") and hasattr(policy, "exploration_noise"):
        mean = np.asarray(policy.mean_action, dtype=np.float32).reshape(ACTION_DIM)
        return _PolicyProgram(N.EVAL_POLICY_SIMPLE, mean, float(policy.exploration_noise),
                              _legacy_global("standard_normal"),
                              lambda s, n: np.random.RandomState(int(s)).standard_normal(n))
    if name == "HeuristicPolicy":
        return _PolicyProgram(N.EVAL_POLICY_HEURISTIC, None, 0.0, _legacy_global("random_sample"),
                              lambda s, n: np.random.RandomState(int(s)).random_sample(n))
    if name == "RandomPolicy" and space is not None:
        return _PolicyProgram(N.EVAL_POLICY_RANDOM, None, 0.0, _generator_doubles(space.np_random),
                              lambda s, n: _pcg(int(s)).random(n))
    raise TypeError(f"{name}: the device evaluator runs the reference's frozen SimpleLearner, HeuristicPolicy and "
                    "RandomPolicy (obs-independent policies)")


# ------------------------------------------------------------------ episode programs
@dataclass
class Segment:
    """One env instance (curriculum row) running consecutive reset(seed) episodes,
    optionally inside CombinedNoiseWrapper(obs_std, dyn_std, seed=noise_seed)."""
    row: int
    episode_seeds: Sequence[Optional[int]]
    obs_std: float = 0.0
    dyn_std: float = 0.0
    noise_seed: Any = None  # None -> entropy (the reference's default_rng(None))


@dataclass
class EvalRecords:
    ep_return: np.ndarray
    ep_length: np.ndarray
    ep_success: np.ndarray
    ep_contacts: np.ndarray
    contact_hist: np.ndarray
    sizes: np.ndarray
    masses: np.ndarray
    frictions: np.ndarray
    policy_used: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))
    obs_traj: Optional[np.ndarray] = None  # f32 [E][max_steps + 1][45] (trajectories=True)
    act_traj: Optional[np.ndarray] = None  # f32 [E][max_steps][15]

    def moments(self) -> HistoryMoments:
        return HistoryMoments.from_padded(self.contact_hist, self.ep_length)


class EpisodeProgram:
    """Host assembly of one ``dxrl_evaluate`` launch: lanes of segments, the
    tapes they consume, the record buffers they fill."""

    def __init__(self, configs: Sequence[Any], reward_type: str = "dense", max_episode_steps: int = 200,
                 max_steps: Optional[int] = None, device=None, reward_shaping=None):
        if len(configs) > N.MAX_CURRICULA:
            raise ValueError(f"at most {N.MAX_CURRICULA} env configurations per launch")
        self.device = device
        self.configs = list(configs)
        self.reward_type, self.reward_shaping = reward_type, reward_shaping
        self.max_episode_steps = int(max_episode_steps)
        self.max_steps = int(max_steps or max_episode_steps)
        self.lanes: List[List[Segment]] = []

    def add_lane(self, segments: Sequence[Segment]):
        self.lanes.append(list(segments))

    @property
    def total_episodes(self) -> int:
        return sum(len(s.episode_seeds) for lane in self.lanes for s in lane)

    def _reset_tape(self, segs):
        tape = np.empty((self.total_episodes, RESET_SLOTS))
        props = np.empty((self.total_episodes, 3))
        k = 0
        for s in segs:
            cfg = self.configs[s.row]
            for j, seed in enumerate(s.episode_seeds):
                tape[k], *p = resolve_reset_draws(_pcg(seed), cfg, first=(j == 0))
                props[k] = [float(x) for x in p]
                k += 1
        return tape, props

    def _constant_props(self, segs):
        props = np.full((self.total_episodes, 3), np.nan)
        k = 0
        for s in segs:
            cfg = self.configs[s.row]
            row = [np.nan if getattr(cfg, r) is not None else float(getattr(cfg, v))
                   for v, r in (("object_size", "object_size_range"), ("object_mass", "object_mass_range"),
                                ("friction_coefficient", "friction_range"))]
            props[k:k + len(s.episode_seeds)] = row
            k += len(s.episode_seeds)
        return props

    def _noise_tape(self, segs):
        """Each noisy segment's wrapper stream: default_rng(seed) standard normals,
        45 per observation-noise draw (reset and step), 15 per dynamics-noise step."""
        chunks, offs, counts, total = [], [], [], 0
        for s in segs:
            o, d = s.obs_std > 0.0, s.dyn_std > 0.0
            if not (o or d):
                offs.append(0)
                counts.append(0)
                continue
            n = len(s.episode_seeds) * (OBS_DIM * o + self.max_steps * (ACTION_DIM * d + OBS_DIM * o))
            chunks.append(np.random.default_rng(s.noise_seed).standard_normal(n))
            offs.append(total)
            counts.append(n)
            total += n
        return (np.concatenate(chunks) if chunks else None), offs, counts

    def plan(self, host_resets: bool = True, host_noise: bool = True) -> "ProgramPlan":
        """Resolve the launch on the host: segment table, lane offsets and the
        parity tapes (no device work; the CPU oracle tests consume this too)."""
        if not self.lanes:
            raise ValueError("no lanes")
        segs = [s for lane in self.lanes for s in lane]
        table = np.zeros(len(segs), dtype=_SEG_DTYPE)
        lane_off = np.zeros(len(self.lanes) + 1, np.int32)
        first = k = 0
        for li, lane in enumerate(self.lanes):
            for s in lane:
                if not 0 <= s.row < len(self.configs):
                    raise ValueError(f"curriculum row {s.row} out of range")
                table[k] = (s.row, len(s.episode_seeds), first, 0, float(s.obs_std), float(s.dyn_std), 0, 0)
                first += len(s.episode_seeds)
                k += 1
            lane_off[li + 1] = k
        noise = None
        if host_noise:
            noise, offs, counts = self._noise_tape(segs)
            table["noise_offset"], table["noise_count"] = offs, counts
        reset, props = self._reset_tape(segs) if host_resets else (None, self._constant_props(segs))
        return ProgramPlan(lane_off, table, reset, props, noise, self.total_episodes)

    def run(self, prog: _PolicyProgram, policy_tapes: Optional[np.ndarray] = None, host_resets: bool = True,
            host_noise: bool = True, device_seed: int = 0, keep_history: bool = True,
            repeat: int = 1, timing: Optional[Dict] = None, trajectories: bool = False) -> EvalRecords:
        """Launch the plan (``repeat`` back-to-back launches; ``timing['kernel_ms']`` =
        HIP-event time per launch on the launch stream)."""
        return self.launch(prog, policy_tapes, host_resets, host_noise, device_seed, keep_history, repeat,
                           trajectories).result(timing)

    def launch(self, prog: _PolicyProgram, policy_tapes: Optional[np.ndarray] = None, host_resets: bool = True,
               host_noise: bool = True, device_seed: int = 0, keep_history: bool = True, repeat: int = 1,
               trajectories: bool = False, stream: Optional[torch.cuda.Stream] = None) -> "_PendingRun":
        """Enqueue the plan on ``stream`` (default: the device's current stream) without waiting;
        ``.result()`` synchronises and returns the records.  Every launch owns its buffers,
        including the work-queue counter, so launches on different streams may overlap."""
        plan = self.plan(host_resets, host_noise)
        dev = self.device = N.require_gpu(self.device)
        nl, E = len(self.lanes), plan.total_episodes
        env = VecEnv(nl, reward_type=self.reward_type, reward_shaping=self.reward_shaping,
                     max_episode_steps=self.max_episode_steps, seed=device_seed, device=dev)
        env.set_curricula(self.configs)
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
        d_lane = t(plan.lane_off, torch.int32)
        d_seg = torch.from_numpy(plan.segments.view(np.uint8).copy()).to(dev)
        mean = None
        if prog.mean is not None:
            mean = t(np.tile(prog.mean, (nl, 1)), torch.float32)
        d_pol = t(policy_tapes, torch.float64) if policy_tapes is not None else None
        d_noise = t(plan.noise, torch.float64) if plan.noise is not None else None
        d_reset = t(plan.reset, torch.float64) if plan.reset is not None else None
        ms = self.max_steps
        out_ret = torch.empty(E, dtype=torch.float64, device=dev)
        out_len = torch.empty(E, dtype=torch.int32, device=dev)
        out_suc = torch.empty(E, dtype=torch.uint8, device=dev)
        out_con = torch.empty(E, dtype=torch.uint8, device=dev)
        out_hist = torch.zeros(E, ms, dtype=torch.uint8, device=dev) if keep_history else None
        used = torch.zeros(nl, dtype=torch.int32, device=dev)
        o_traj = torch.zeros(E, ms + 1, OBS_DIM, dtype=torch.float32, device=dev) if trajectories else None
        a_traj = torch.zeros(E, ms, ACTION_DIM, dtype=torch.float32, device=dev) if trajectories else None
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        queue = torch.zeros(1, dtype=torch.int32, device=dev)  # this launch's work-queue counter
        a = N.EvalArgs()
        a.num_lanes, a.policy, a.max_steps, a.total_episodes = nl, prog.kind, ms, E
        a.lane_segments, a.segments, a.mean_action = N.ptr(d_lane), N.ptr(d_seg), N.ptr(mean)
        a.exploration_noise = prog.sigma
        a.policy_tape = N.ptr(d_pol)
        a.policy_stride = 0 if policy_tapes is None else policy_tapes.shape[1]
        a.noise_tape, a.reset_tape = N.ptr(d_noise), N.ptr(d_reset)
        a.policy_seed = a.noise_seed = a.reset_seed = int(device_seed) & (2**64 - 1)
        a.ep_return, a.ep_length, a.ep_success = N.ptr(out_ret), N.ptr(out_len), N.ptr(out_suc)
        a.ep_contacts, a.contact_hist = N.ptr(out_con), N.ptr(out_hist)
        a.policy_used, a.status = N.ptr(used), N.ptr(status)
        a.obs_traj, a.act_traj, a.work_queue = N.ptr(o_traj), N.ptr(a_traj), N.ptr(queue)
        with torch.cuda.device(dev):
            st = stream if stream is not None else torch.cuda.current_stream(dev)
            # the inputs were written on the current stream; the launch stream waits for them
            st.wait_stream(torch.cuda.current_stream(dev))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(max(1, int(repeat))):
                N.call("dxrl_evaluate", env.handle, C.byref(a), st.cuda_stream)
            e1.record(st)
        keep = (env, a, d_lane, d_seg, mean, d_pol, d_noise, d_reset, queue)  # alive until the stream is done
        outs = (out_ret, out_len, out_suc, out_con, out_hist, used, o_traj, a_traj)
        if st != torch.cuda.current_stream(dev):
            # allocated on the current stream, used on `st`: the caching allocator must not hand
            # these blocks out again before `st` has passed the launch, even if the _PendingRun
            # is dropped without result()
            for x in outs + (status, d_lane, d_seg, mean, d_pol, d_noise, d_reset, queue, env._slab_owner):
                if isinstance(x, torch.Tensor):
                    x.record_stream(st)
        return _PendingRun(st, e0, e1, max(1, int(repeat)), status, plan.props, keep_history, trajectories, outs,
                           keep, E)


    def run_facade(self, policy, trajectories: bool = False) -> EvalRecords:
        """The plan's episodes in order through the Gymnasium facade (one device env step per
        call) with a host policy -- the path for policies the kernel does not compile (any
        ``select_action``), running evaluator.py:71-181 / robustness_tests.py:262-303 as
        written: a fresh env per segment, CombinedNoiseWrapper when the segment is noisy."""
        from .envs import DexterousManipulationEnv
        from .evaluation import CombinedNoiseWrapper
        E, ms = self.total_episodes, self.max_steps
        ret, length = np.zeros(E), np.zeros(E, np.int32)
        succ, cont = np.zeros(E, bool), np.zeros(E, np.uint8)
        hist, props = np.zeros((E, ms), np.uint8), np.full((E, 3), np.nan)
        otraj = np.zeros((E, ms + 1, OBS_DIM), np.float32) if trajectories else None
        atraj = np.zeros((E, ms, ACTION_DIM), np.float32) if trajectories else None
        k = 0
        for seg in (s for lane in self.lanes for s in lane):
            base = DexterousManipulationEnv(curriculum_config=self.configs[seg.row], reward_type=self.reward_type,
                                            reward_shaping=self.reward_shaping,
                                            max_episode_steps=self.max_episode_steps, device=self.device)
            noisy = seg.obs_std > 0.0 or seg.dyn_std > 0.0
            env = CombinedNoiseWrapper(base, seg.obs_std, seg.dyn_std, seed=seg.noise_seed) if noisy else base
            for seed in seg.episode_seeds:
                obs, info = env.reset(seed=seed)
                if hasattr(policy, "reset"):
                    policy.reset()
                if trajectories:
                    otraj[k, 0] = obs
                total, te, n = 0.0, False, 0
                for step in range(ms):
                    a = policy.select_action(obs)
                    if trajectories:
                        atraj[k, step] = a
                    obs, r, te, tr, info = env.step(a)
                    total += r
                    n = step + 1
                    hist[k, step] = info.get("num_contacts", 0)
                    if trajectories:
                        otraj[k, step + 1] = obs
                    if te or tr:
                        break
                ret[k], length[k], succ[k], cont[k] = total, n, bool(te), info.get("num_contacts", 0)
                c = info["curriculum"]
                props[k] = [c["object_size"], c["object_mass"], c["friction_coefficient"]]
                k += 1
            env.close()
        return EvalRecords(ret, length, succ, cont, hist, props[:, 0], props[:, 1], props[:, 2],
                           np.zeros(len(self.lanes), np.int32), otraj, atraj)


_SEG_DTYPE = np.dtype([("curriculum_row", "<i4"), ("num_episodes", "<i4"), ("first_episode", "<i4"),
                       ("reserved", "<i4"), ("obs_noise_std", "<f8"), ("dyn_noise_std", "<f8"),
                       ("noise_offset", "<i8"), ("noise_count", "<i8")])


@dataclass
class ProgramPlan:
    lane_off: np.ndarray          # i32 [lanes + 1]
    segments: np.ndarray          # _SEG_DTYPE [segments] == dxrl_eval_segment
    reset: Optional[np.ndarray]   # f64 [E][D+6] or None (device Philox resets)
    props: np.ndarray             # f64 [E][3] size, mass, friction of each episode (NaN: device-drawn)
    noise: Optional[np.ndarray]   # f64 standard normals or None (device Philox noise)
    total_episodes: int


class _PendingRun:
    """An enqueued dxrl_evaluate launch (EpisodeProgram.launch); result() waits for its stream."""

    def __init__(self, stream, e0, e1, repeat, status, props, keep_history, trajectories, outs, keep, E):
        self.stream, self.e0, self.e1, self.repeat = stream, e0, e1, repeat
        self.status, self.props, self.keep_history, self.trajectories = status, props, keep_history, trajectories
        self.outs, self.keep, self.E = outs, keep, E

    def result(self, timing: Optional[Dict] = None) -> EvalRecords:
        self.stream.synchronize()
        if timing is not None:
            timing["kernel_ms"] = self.e0.elapsed_time(self.e1) / self.repeat
        if int(self.status.item()):
            raise N.NativeError("dxrl_evaluate: a parity tape ran out or a segment was malformed")
        self.keep[0].close()
        out_ret, out_len, out_suc, out_con, out_hist, used, o_traj, a_traj = self.outs
        p = self.props
        return EvalRecords(out_ret.cpu().numpy(), out_len.cpu().numpy(), out_suc.cpu().numpy().astype(bool),
                           out_con.cpu().numpy(),
                           out_hist.cpu().numpy() if self.keep_history else np.zeros((self.E, 0), np.uint8),
                           p[:, 0], p[:, 1], p[:, 2], used.cpu().numpy(),
                           o_traj.cpu().numpy() if self.trajectories else None,
                           a_traj.cpu().numpy() if self.trajectories else None)


def _exact_tape(prog: _PolicyProgram, program: EpisodeProgram) -> np.ndarray:
    need = program.total_episodes * program.max_steps * ACTION_DIM
    if need > _MAX_TAPE:
        raise ValueError(f"exact-order evaluation would need a {need}-draw policy tape; use parallel=True")
    return prog.stream.draw(need)[None, :]


def _seeded_tapes(prog: _PolicyProgram, program: EpisodeProgram, policy_seeds) -> np.ndarray:
    if len(policy_seeds) != len(program.lanes):
        raise ValueError("one policy seed per episode")
    return np.stack([prog.seeded(s, program.max_steps * ACTION_DIM) for s in policy_seeds])


def _episode_dicts(rec: EvalRecords, idx: np.ndarray, with_props: bool) -> List[Dict]:
    out = []
    for i in idx:
        n = int(rec.ep_length[i])
        hist = rec.contact_hist[i, :n] if rec.contact_hist.shape[1] else np.zeros(0, np.uint8)
        d = {"episode_reward": float(rec.ep_return[i]), "episode_steps": n, "success": bool(rec.ep_success[i]),
             "num_contacts": int(rec.ep_contacts[i]), "final_contacts": int(rec.ep_contacts[i]),
             "contact_history": [[1.0 if j < c else 0.0 for j in range(5)] for c in hist.tolist()]}
        if with_props:
            d["object_size"], d["object_mass"], d["friction_coefficient"] = (
                float(rec.sizes[i]), float(rec.masses[i]), float(rec.frictions[i]))
        out.append(d)
    return out


def _metrics(rec: EvalRecords, idx: np.ndarray, max_steps: int) -> Dict:
    m = rec.moments()
    sel = lambda x: np.asarray(x)[idx]  # noqa: E731
    sub = HistoryMoments(sel(m.n), sel(m.s1), sel(m.s2), sel(m.first5), sel(m.last5), lambda i: m.row(idx[i]))
    codes = classify_columns(sel(rec.ep_success), sel(rec.ep_length), sel(rec.ep_contacts), sel(rec.ep_contacts),
                             sub, max_steps, 3)
    return aggregate_columns(sel(rec.ep_success), sel(rec.ep_length), sel(rec.ep_contacts), codes)


# ------------------------------------------------------------------ Evaluator
class Evaluator:
    """evaluation/evaluator.py:17-271 on the device."""

    def __init__(self, policy, heldout_set, reward_type: str = "dense", max_episode_steps: int = 200,
                 failure_logger=None, device=None):
        self.policy = policy
        self.heldout_set = heldout_set
        self.reward_type = reward_type
        self.max_episode_steps = max_episode_steps
        self.failure_logger = failure_logger
        self.device = device
        self._policy_frozen = False

    # evaluator.py:50-69
    def freeze_policy(self):
        if hasattr(self.policy, "update"):
            self._original_update = self.policy.update
            self.policy.update = lambda *a, **k: None
            self._policy_frozen = True

    def unfreeze_policy(self):
        if self._policy_frozen and hasattr(self, "_original_update"):
            self.policy.update = self._original_update
            self._policy_frozen = False

    def __enter__(self):
        self.freeze_policy()
        return self

    def __exit__(self, exc_type, exc, tb):
        self.unfreeze_policy()

    def _program(self, configs):
        return EpisodeProgram(configs, self.reward_type, self.max_episode_steps, device=self.device)

    def evaluate_episode(self, eval_config, seed: Optional[int] = None) -> Dict:
        """evaluator.py:71-181: one episode on a fresh env instance."""
        if not self._policy_frozen:
            self.freeze_policy()
        prog = compiled_program(self.policy)
        p = self._program([eval_config])
        p.add_lane([Segment(0, [seed])])
        traj = self.failure_logger is not None
        if prog is None:
            rec = p.run_facade(self.policy, trajectories=traj)
        else:
            rec = p.run(prog, policy_tapes=_exact_tape(prog, p), trajectories=traj)
            prog.stream.commit(int(rec.policy_used[0]))
        out = _episode_dicts(rec, np.arange(1), True)
        self._log_failures(rec, out, [eval_config], [seed])
        return out[0]

    def _log_failures(self, rec: EvalRecords, episodes: List[Dict], configs, seeds):
        """evaluator.py:101-179: EpisodeRecorder contents of each failed episode -> failure_logger."""
        if self.failure_logger is None:
            return
        for i, ep in enumerate(episodes):
            if ep["success"]:
                continue
            n = ep["episode_steps"]
            cfg = configs[i]
            cfg_dict = cfg.to_dict() if hasattr(cfg, "to_dict") else {
                "object_size": cfg.object_size, "object_mass": cfg.object_mass,
                "friction_coefficient": cfg.friction_coefficient}
            states = [rec.obs_traj[i, k].copy() for k in range(n + 1)]
            c0 = int(rec.obs_traj[i, 0, 40:45].sum())  # info["num_contacts"] after reset
            contacts = [[1.0 if j < c0 else 0.0 for j in range(5)]] + ep["contact_history"]
            meta = {"seed": seeds[i], "eval_config": cfg_dict, "object_size": ep["object_size"],
                    "object_mass": ep["object_mass"], "friction_coefficient": ep["friction_coefficient"]}
            self.failure_logger.log_episode(episode_data=ep, states=states,
                                            actions=[rec.act_traj[i, k].copy() for k in range(n)],
                                            contacts=contacts, metadata=meta, max_steps=self.max_episode_steps)

    def heldout_program(self, num_episodes_per_object: int, seed: Optional[int], parallel: bool) -> EpisodeProgram:
        """The launch plan of evaluate_heldout_set: object-major episodes (object i,
        episode k -> record i*K + k) with reset seed ``seed + k`` (or default_rng(None)
        draws, evaluator.py:210-213); one lane in exact order, one lane per episode
        when parallel."""
        objs = self.heldout_set.heldout_objects
        n_obj, K = len(objs), int(num_episodes_per_object)
        configs = [self.heldout_set.get_eval_config(i) for i in range(n_obj)]
        rng = np.random.default_rng(seed)
        seeds = [[(int(rng.integers(0, 2**31)) if seed is None else seed + e) for e in range(K)]
                 for _ in range(n_obj)]
        p = self._program(configs)
        if not parallel:
            p.add_lane([Segment(o, [seeds[o][e]]) for o in range(n_obj) for e in range(K)])
        else:
            for o in range(n_obj):
                for e in range(K):
                    p.add_lane([Segment(o, [seeds[o][e]])])
        return p

    def evaluate_heldout_set(self, num_episodes_per_object: int = 5, seed: Optional[int] = None,
                             parallel: bool = False, policy_seeds: Optional[Sequence[int]] = None,
                             device_seed: int = 0, return_episodes: bool = True) -> Dict:
        """evaluator.py:183-262 (see heldout_program for the episode layout)."""
        if not self._policy_frozen:
            self.freeze_policy()
        prog = compiled_program(self.policy)
        p = self.heldout_program(num_episodes_per_object, seed, parallel and prog is not None)
        traj = self.failure_logger is not None
        if prog is None:  # host policy: the reference's sequential loop on the facade
            rec = p.run_facade(self.policy, trajectories=traj)
        elif not parallel:
            rec = p.run(prog, policy_tapes=_exact_tape(prog, p), trajectories=traj)
            prog.stream.commit(int(rec.policy_used[0]))
        elif policy_seeds is not None:
            rec = p.run(prog, policy_tapes=_seeded_tapes(prog, p, policy_seeds), trajectories=traj)
        else:
            rec = p.run(prog, host_resets=False, host_noise=False, device_seed=device_seed, trajectories=traj)
        res = self.results(rec, int(num_episodes_per_object), return_episodes or traj)
        if traj:
            segs = [lane_seg for lane in p.lanes for lane_seg in lane]
            self._log_failures(rec, res["all_episodes"], [p.configs[s.row] for s in segs],
                               [s.episode_seeds[0] for s in segs])
        return res

    def results(self, rec: EvalRecords, K: int, return_episodes: bool = True) -> Dict:
        """evaluator.py:229-262 result dicts from the episode records."""
        objs = self.heldout_set.heldout_objects
        n_obj = len(objs)
        ms = self.max_episode_steps
        E = n_obj * K
        all_idx = np.arange(E)
        all_eps = _episode_dicts(rec, all_idx, True) if return_episodes else None
        if all_eps is not None:
            for i, d in enumerate(all_eps):
                d["object_idx"], d["episode"] = i // K, i % K
        per_object = {}
        per_object_metrics = {}
        for o in range(n_obj):
            idx = np.arange(o * K, (o + 1) * K)
            entry = {"object_properties": {"size": objs[o].size, "mass": objs[o].mass, "friction": objs[o].friction}}
            if all_eps is not None:
                entry["episodes"] = all_eps[o * K:(o + 1) * K]
            entry["mean_reward"] = float(np.mean(rec.ep_return[idx]))
            entry["mean_steps"] = float(np.mean(rec.ep_length[idx].astype(np.int64)))
            entry["success_rate"] = float(np.mean(np.where(rec.ep_success[idx], 1.0, 0.0)))
            per_object[o] = entry
            if K:
                per_object_metrics[o] = _metrics(rec, idx, ms)
        agg = _metrics(rec, all_idx, ms) if E else {}
        overall = {"num_objects": n_obj, "total_episodes": E,
                   "overall_success_rate": agg.get("grasp_success_rate"),
                   "mean_reward": float(np.mean(rec.ep_return)), "std_reward": float(np.std(rec.ep_return)),
                   "mean_steps": agg.get("mean_episode_length")}
        out = {"overall_stats": overall, "per_object_results": per_object, "all_episodes": all_eps,
               "metrics": agg, "per_object_metrics": per_object_metrics}
        if not return_episodes:
            out["records"] = rec
        return out


# ------------------------------------------------------------------ RobustnessTester
class RobustnessTester:
    """evaluation/robustness_tests.py:212-407 on the device."""

    def __init__(self, policy, eval_config, reward_type: str = "dense", max_episode_steps: int = 200, device=None):
        self.policy = policy
        self.eval_config = eval_config
        self.reward_type = reward_type
        self.max_episode_steps = max_episode_steps
        self.device = device

    def _level_segment(self, obs: float, dyn: float, num_episodes: int, seed: Optional[int]) -> Segment:
        rng = np.random.default_rng(seed)  # robustness_tests.py:276-281
        seeds = [(int(rng.integers(0, 2**31)) if seed is None else seed + e) for e in range(num_episodes)]
        return Segment(0, seeds, obs, dyn, noise_seed=seed)

    @staticmethod
    def sweep_levels(observation_noise_levels, dynamics_noise_levels):
        """robustness_tests.py:333-405 level order: baseline, observation levels,
        dynamics levels, then the first-three x first-three combinations."""
        levels, keys = [(0.0, 0.0)], [("baseline", None)]
        for o in observation_noise_levels:
            if o > 0.0:
                levels.append((o, 0.0))
                keys.append(("observation_noise", o))
        for d in dynamics_noise_levels:
            if d > 0.0:
                levels.append((0.0, d))
                keys.append(("dynamics_noise", d))
        for o in observation_noise_levels[:3]:
            for d in dynamics_noise_levels[:3]:
                if o > 0.0 or d > 0.0:
                    levels.append((o, d))
                    keys.append(("combined_noise", f"obs_{o:.3f}_dyn_{d:.3f}"))
        return levels, keys

    def levels_program(self, levels, num_episodes: int, seed: Optional[int], parallel: bool) -> EpisodeProgram:
        """One segment per noise level (a fresh base env, CombinedNoiseWrapper(seed)
        when a level is noisy, robustness_tests.py:266-278); exact order = one lane
        through all levels, parallel = one lane (fresh env) per episode."""
        p = EpisodeProgram([self.eval_config], self.reward_type, self.max_episode_steps, device=self.device)
        segs = [self._level_segment(o, d, num_episodes, seed) for o, d in levels]
        if not parallel:
            p.add_lane(segs)
        else:
            for s in segs:
                for k, es in enumerate(s.episode_seeds):
                    p.add_lane([Segment(0, [es], s.obs_std, s.dyn_std,
                                        noise_seed=None if s.noise_seed is None else (s.noise_seed, k))])
        return p

    def _run_levels(self, levels, num_episodes, seed, parallel, policy_seeds, device_seed):
        prog = compiled_program(self.policy)
        p = self.levels_program(levels, num_episodes, seed, parallel and prog is not None)
        if prog is None:  # host policy: the reference's sequential loop on the facade
            rec = p.run_facade(self.policy)
        elif not parallel:
            rec = p.run(prog, policy_tapes=_exact_tape(prog, p))
            prog.stream.commit(int(rec.policy_used[0]))
        elif policy_seeds is not None:
            rec = p.run(prog, policy_tapes=_seeded_tapes(prog, p, policy_seeds))
        else:
            rec = p.run(prog, host_resets=False, host_noise=False, device_seed=device_seed)
        return self.level_results(rec, levels, num_episodes)

    def level_results(self, rec: EvalRecords, levels, num_episodes: int) -> List[Dict]:
        """robustness_tests.py:296-310 result dicts, one per level."""
        out = []
        for li, (o, d) in enumerate(levels):
            idx = np.arange(li * num_episodes, (li + 1) * num_episodes)
            eps = []
            for e in _episode_dicts(rec, idx, False):  # robustness_tests.py:296-303 key order
                e["episode_reward"] = e.pop("episode_reward")
                eps.append(e)
            out.append({"episodes": eps, "metrics": _metrics(rec, idx, self.max_episode_steps) if len(idx) else {},
                        "noise_levels": {"observation_noise_std": o, "dynamics_noise_std": d}})
        return out

    def evaluate_with_noise(self, observation_noise_std: float = 0.0, dynamics_noise_std: float = 0.0,
                            num_episodes: int = 20, seed: Optional[int] = None, parallel: bool = False,
                            policy_seeds: Optional[Sequence[int]] = None, device_seed: int = 0) -> Dict:
        """robustness_tests.py:240-310."""
        return self._run_levels([(observation_noise_std, dynamics_noise_std)], num_episodes, seed, parallel,
                                policy_seeds, device_seed)[0]

    def run_robustness_sweep(self, observation_noise_levels: List[float], dynamics_noise_levels: List[float],
                             num_episodes: int = 20, seed: Optional[int] = None, parallel: bool = False,
                             policy_seeds: Optional[Sequence[int]] = None, device_seed: int = 0) -> Dict:
        """robustness_tests.py:312-407: every level of the sweep as a segment of one launch."""
        levels, keys = self.sweep_levels(observation_noise_levels, dynamics_noise_levels)
        res = self._run_levels(levels, num_episodes, seed, parallel, policy_seeds, device_seed)
        out: Dict[str, Any] = {"baseline": None, "observation_noise": {}, "dynamics_noise": {}, "combined_noise": {}}
        for (grp, k), r in zip(keys, res):
            if grp == "baseline":
                out["baseline"] = r
            else:
                out[grp][k] = r
        return out


__all__ = ["Evaluator", "RobustnessTester", "EpisodeProgram", "Segment", "EvalRecords", "EvaluationMetrics",
           "policy_program", "failure_names"]
