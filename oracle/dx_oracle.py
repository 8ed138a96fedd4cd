"""CPU oracle: scalar NumPy restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product (the HIP library behind
``include/dxrl.h``) never calls it and has no CPU fallback.

Parity: PINNED.  ``tests/test_oracle_golden.py`` checks this restatement
bit-exactly (obs, flags, contacts, object position, learner state) and to
1e-12 relative on rewards (np.exp vs libm differ by <= 1 ulp) against the
fixtures in ``tests/golden/`` that ``tests/golden/gen_golden.py`` captured
from the reference itself.

Each function follows the reference op by op under NumPy 2 / NEP 50 scalar
promotion:

* ``OracleEnv.reset``  <- envs/manipulation_env.py:124-182, experiments/config.py:44-113
* ``OracleEnv.step``   <- envs/manipulation_env.py:184-252
* ``_contacts``        <- envs/manipulation_env.py:285-310
* ``_dense_reward``    <- rewards/reward_shaping.py:50-187
* ``_sparse_reward``   <- rewards/reward_shaping.py:205-242
* ``OracleSimpleLearner`` <- policies/simple_learner.py:49-99
* ``oracle_run_episode``  <- training/episode_utils.py:13-55
* ``oracle_eval_program`` <- evaluation/evaluator.py:71-181, robustness_tests.py:240-310
  (pinned by tests/test_eval_host.py against tests/golden/eval_golden.json)

Throughput-mode RNG (the build's own, not the reference's: the reference draws reset
values from gymnasium's PCG64, which the device replaces with per-env Philox4x32-10
streams -- distributional parity only, SURVEY.md §7 "RNG parity"):

* ``philox4x32_10`` / ``env_key`` / ``philox_reset_draws`` restate csrc/dxrl_device.h
  (philox, env_key, env_reset_philox) so the full-size rollout tests can replay a lane's
  auto-resets.  Pinned by the Random123 known-answer vectors for philox4x32-10
  (tests/test_oracle_golden.py::test_philox_known_answers).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

f32 = np.float32
F, J, D = 5, 3, 15
LO = (-0.2, -0.2, 0.0)   # manipulation_env.py:119 workspace bounds
HI = (0.2, 0.2, 0.3)
GZ = -9.81 * 0.01        # manipulation_env.py:211-212 (f64)


@dataclass
class OracleCurriculum:
    """experiments/config.py:17-42 (only what reset/step read)."""
    object_size: float = 0.05
    object_mass: float = 0.1
    friction_coefficient: float = 0.5
    size_range: Optional[Sequence[float]] = None
    mass_range: Optional[Sequence[float]] = None
    friction_range: Optional[Sequence[float]] = None
    spawn_x_range: Sequence[float] = (-0.1, 0.1)
    spawn_y_range: Sequence[float] = (-0.1, 0.1)
    spawn_z_range: Sequence[float] = (0.05, 0.2)
    # NEP 50: a numpy.float64 friction (scheduler interpolation) makes
    # `ov *= damping` an f64 multiply instead of an f32 one.
    friction_is_np_float64: bool = False

    @classmethod
    def from_record(cls, r: dict) -> "OracleCurriculum":
        return cls(object_size=r["object_size"], object_mass=r["object_mass"],
                   friction_coefficient=r["friction_coefficient"],
                   size_range=r.get("object_size_range"), mass_range=r.get("object_mass_range"),
                   friction_range=r.get("friction_range"),
                   spawn_x_range=r["spawn_x_range"], spawn_y_range=r["spawn_y_range"],
                   spawn_z_range=r["spawn_z_range"],
                   friction_is_np_float64="friction_coefficient" in r.get("_float64_scalars", []))


def reset_draws(rng: np.random.Generator, cur: OracleCurriculum, first: bool) -> np.ndarray:
    """The 21 draw slots reset() consumes, in the reference's order
    (manipulation_env.py:143-161); NaN where no draw happens."""
    jp = rng.uniform(low=-0.1, high=0.1, size=(D,))
    size = mass = fric = math.nan
    if cur.size_range is not None:
        size = float(rng.uniform(cur.size_range[0], cur.size_range[1]))
    if cur.mass_range is not None:
        mass = float(rng.uniform(cur.mass_range[0], cur.mass_range[1]))
    if cur.friction_range is not None:
        fric = float(rng.uniform(cur.friction_range[0], cur.friction_range[1]))
    spawn = [math.nan] * 3
    if first:
        spawn = [float(rng.uniform(*cur.spawn_x_range)), float(rng.uniform(*cur.spawn_y_range)),
                 float(rng.uniform(*cur.spawn_z_range))]
    return np.concatenate([jp, [size, mass, fric], spawn])


def _clip(x, lo, hi):
    return lo if x < lo else (hi if x > hi else x)


@dataclass
class OracleEnv:
    """One DexterousManipulationEnv, scalar state in exact reference dtypes."""
    cur: OracleCurriculum = field(default_factory=OracleCurriculum)
    dense: bool = True
    max_episode_steps: int = 200
    weights: Sequence[float] = (1.0, 0.5, 0.3, 0.2)  # reward_shaping.py:22-25
    object_position: Optional[Sequence[float]] = None  # constructor arg (:28)

    def __post_init__(self):
        self.jp = [f32(0)] * D
        self.jv = [f32(0)] * D
        self.op = None if self.object_position is None else [float(v) for v in self.object_position]
        self.op_is_f32 = True
        self.ov = [f32(0)] * 3
        self.contacts = [0] * F
        self.prev = None
        self.t = 0
        self.size = self.mass = self.fric = None
        self.last_components = None

    # -- A2 ---------------------------------------------------------------
    def reset(self, draws: np.ndarray):
        self.jp = [f32(v) for v in draws[:D]]
        self.jv = [f32(0)] * D
        c = self.cur
        self.size = draws[D] if c.size_range is not None else c.object_size
        self.mass = draws[D + 1] if c.mass_range is not None else c.object_mass
        self.fric = draws[D + 2] if c.friction_range is not None else c.friction_coefficient
        if self.op is None:
            src = draws[D + 3:D + 6]
        else:
            src = self.op
        self.op = [float(f32(v)) for v in src]  # np.array(..., dtype=float32)
        self.op_is_f32 = True
        self.ov = [f32(0)] * 3
        self.t = 0
        self._contacts()
        self.prev = None
        return self.obs()

    # -- A4 ---------------------------------------------------------------
    def _contacts(self):
        thr = self.size * 1.5
        self.tips, self.dist = [], []
        for f in range(F):
            s = f32(f32(self.jp[3 * f] + self.jp[3 * f + 1]) + self.jp[3 * f + 2])
            tip = float(f32(s * f32(0.1)))
            dx, dy, dz = tip - self.op[0], tip - self.op[1], tip - self.op[2]
            d = math.sqrt((dx * dx + dy * dy) + dz * dz)
            self.tips.append(tip)
            self.dist.append(d)
        self.contacts = [1 if d < thr else 0 for d in self.dist]

    # -- A5 / A6 -----------------------------------------------------------
    def _dense_reward(self):
        dist = float(np.exp(-5.0 * min(self.dist)))
        n = sum(self.contacts)
        con = n / F
        cl = []
        for f in range(F):
            acc = f32(0)
            for j in range(J):
                v = self.jp[3 * f + j]
                if v < 0:
                    acc = f32(acc + v)
            cl.append(f32(-acc))
        s = f32(0)
        for v in cl:
            s = f32(s + v)
        avg = f32(s / f32(F))
        clo = float(_clip(f32(avg / f32(F)), f32(0), f32(1)))
        if self.prev is None:
            self.prev = list(self.contacts)
            st = 0.0
        else:
            ch = f32(0)
            for a, b in zip(self.contacts, self.prev):
                ch = f32(ch + f32(abs(a - b)))
            st = float(_clip(f32(f32(1) - f32(ch / f32(F))), f32(0), f32(1)))
            self.prev = list(self.contacts)
        w = self.weights
        total = w[0] * dist + w[1] * con + w[2] * clo + w[3] * st
        return total, (dist, con, clo, st)

    def _sparse_reward(self):
        return (1.0 if sum(self.contacts) >= 3 else -0.01), (0.0, 0.0, 0.0, 0.0)

    # -- A3 + A7 -----------------------------------------------------------
    def step(self, action):
        a = [_clip(f32(x), f32(-1), f32(1)) for x in action]
        self.jv = [f32(f32(f32(0.9) * v) + f32(f32(0.1) * x)) for v, x in zip(self.jv, a)]
        self.jp = [_clip(f32(p + f32(v * f32(0.01))), f32(-1), f32(1)) for p, v in zip(self.jp, self.jv)]
        damp = 1.0 - (self.fric * 0.1 * 0.01)
        if self.cur.friction_is_np_float64:
            self.ov = [f32(float(v) * damp) for v in self.ov]
        else:
            self.ov = [f32(v * f32(damp)) for v in self.ov]
        self.ov = [f32(float(v) + g) for v, g in zip(self.ov, (0.0, 0.0, GZ))]
        inc = [f32(v * f32(0.01)) for v in self.ov]
        if self.op_is_f32:
            op = [float(f32(f32(p) + i)) for p, i in zip(self.op, inc)]
        else:
            op = [p + float(i) for p, i in zip(self.op, inc)]
        self.op = [min(max(p, lo), hi) for p, lo, hi in zip(op, LO, HI)]
        self.op_is_f32 = False
        for i in range(3):
            if (self.op[i] <= LO[i] and self.ov[i] < 0) or (self.op[i] >= HI[i] and self.ov[i] > 0):
                self.ov[i] = f32(0)
        self._contacts()
        reward, comps = self._dense_reward() if self.dense else self._sparse_reward()
        self.last_components = comps
        n = sum(self.contacts)
        terminated = n >= 3
        truncated = self.t >= self.max_episode_steps
        self.t += 1
        return self.obs(), reward, terminated, truncated

    def obs(self):
        o = np.empty(45, np.float32)
        o[0:15] = self.jp
        o[15:30] = self.jv
        o[30:33] = self.op
        o[33:37] = (1.0, 0.0, 0.0, 0.0)
        o[37:40] = self.ov
        o[40:45] = self.contacts
        return o

    @property
    def num_contacts(self):
        return sum(self.contacts)


class OracleSimpleLearner:
    """policies/simple_learner.py:13-99 driven by a tape of legacy-MT19937
    gauss values (np.random.normal(0, s) == 0 + s * gauss)."""

    def __init__(self, gauss: np.ndarray, learning_rate=0.01, exploration_noise=0.3, clip_range=0.5):
        self.g = gauss
        self.cur = 0
        self.lr, self.noise, self.clip = learning_rate, exploration_noise, clip_range
        self.mean = [f32(0)] * D
        self.best = -math.inf

    def _take(self, n):
        v = self.g[self.cur:self.cur + n]
        self.cur += n
        return v

    def select_action(self):
        g = self._take(D)
        return [_clip(f32(m + f32(0.0 + self.noise * x)), f32(-1), f32(1)) for m, x in zip(self.mean, g)]

    def update(self, reward):
        if reward > self.best:
            g = self._take(D)
            self.mean = [_clip(f32(float(m) + (0.0 + self.lr * x)), f32(-self.clip), f32(self.clip))
                         for m, x in zip(self.mean, g)]
            self.best = reward

    def reset(self):
        self.best = -math.inf


def oracle_run_episode(env: OracleEnv, pol: OracleSimpleLearner, draws, max_steps=None):
    """training/episode_utils.py:13-55 with the training-loop success rule
    (info has no "success" key, :52) -> success is always False."""
    env.reset(draws)
    pol.reset()
    max_steps = max_steps or env.max_episode_steps
    total = 0.0
    step = 0
    for step in range(max_steps):
        a = pol.select_action()
        _, r, term, trunc = env.step(a)
        total += r
        pol.update(r)
        if term or trunc:
            break
    return False, step + 1, total


def oracle_noisy_action(action, noise):
    """evaluation/robustness_tests.py:180-187: a' = clip(a + f32(n), low, high)."""
    return [_clip(f32(f32(a) + f32(n)), f32(-1), f32(1)) for a, n in zip(action, noise)]


def oracle_noisy_obs(obs, noise):
    """evaluation/robustness_tests.py:199-207: obs + f32(n) (f32 add)."""
    return (obs + np.asarray(noise).astype(np.float32)).astype(np.float32)


# ---------------------------------------------------------------- reward plugins on given inputs
def oracle_reward_compute(joint_positions, finger_tips, object_position, contacts, prev_contacts, weights,
                          dense: bool = True, num_fingers: int = F, joints_per_finger: int = J):
    """RewardShaping.compute (rewards/reward_shaping.py:50-187) / SparseReward.compute (:205-242)
    on caller-given arrays, with numpy's own functions in the reference's dtypes (f32 joints and
    contacts, f64 tips and object position).  Returns ((total, distance, contact, closure,
    stability), new prev_contacts); prev_contacts None = the first call after reset()."""
    c = np.asarray(contacts, np.float32)
    n_con = np.sum(c > 0.5)
    if not dense:
        return ((1.0 if n_con >= 3 else -0.01), 0.0, 0.0, 0.0, 0.0), prev_contacts
    jp = np.asarray(joint_positions, np.float32)
    d = np.linalg.norm(np.asarray(finger_tips, np.float64) - np.asarray(object_position, np.float64), axis=1)
    dist = float(np.exp(-5.0 * np.min(d)))                        # :111-118
    con = float(n_con / num_fingers)                               # :130-136
    scores = []
    for f in range(num_fingers):                                   # :149-164
        fj = jp[f * joints_per_finger:(f + 1) * joints_per_finger]
        scores.append(-np.sum(fj[fj < 0]))
    clo = float(np.clip(np.mean(scores) / num_fingers, 0.0, 1.0))
    if prev_contacts is None:                                      # :172-175
        st = 0.0
    else:                                                          # :178-187
        ch = np.sum(np.abs(c - np.asarray(prev_contacts, np.float32)))
        st = float(np.clip(1.0 - (ch / len(c)), 0.0, 1.0))
    w = weights
    total = w[0] * dist + w[1] * con + w[2] * clo + w[3] * st     # :86-91
    return (total, dist, con, clo, st), c.copy()


def oracle_finger_tips(jp):
    """envs/manipulation_env.py:296-303: tip_f = zeros(3) + f32(sum(joints of f)) * 0.1 -> f64 [5][3]."""
    jp = np.asarray(jp, np.float32)
    out = np.empty((F, 3), np.float64)
    for f in range(F):
        out[f] = np.array([0.0, 0.0, 0.0]) + np.sum(jp[f * J:(f + 1) * J]) * 0.1
    return out


# ---------------------------------------------------------------- evaluation episode programs
POLICY_SIMPLE, POLICY_HEURISTIC, POLICY_RANDOM = 0, 1, 2


def oracle_policy_action(kind: int, mean, sigma: float, draws):
    """One frozen-policy action from 15 raw draws:
    SimpleLearner  clip(mean + f32(0 + s g), -1, 1)           (simple_learner.py:59-71)
    Heuristic      clip(f32(-0.5) + f32(-0.1 + 0.2 u), -1, 1)   (heuristic_policy.py:51-63)
    Random         f32(-1 + 2 u)  (Box.sample: uniform(low, high).astype(f32))"""
    if kind == POLICY_SIMPLE:
        return [_clip(f32(m + f32(0.0 + sigma * g)), f32(-1), f32(1)) for m, g in zip(mean, draws)]
    if kind == POLICY_HEURISTIC:
        return [_clip(f32(f32(-0.5) + f32(-0.1 + (0.1 - -0.1) * u)), f32(-1), f32(1)) for u in draws]
    return [f32(-1.0 + (1.0 - -1.0) * u) for u in draws]


def oracle_eval_program(curricula, lane_off, segments, reset_tape, policy_tapes, noise_tape, kind: int, mean,
                        sigma: float, max_steps: int, dense: bool = True, max_episode_steps: int = 200):
    """Restates the evaluation drivers' episode loops (evaluation/evaluator.py:71-181 per
    episode on a fresh env; robustness_tests.py:240-310 consecutive episodes on one
    env inside CombinedNoiseWrapper) for a lane/segment plan (include/dxrl.h
    dxrl_eval_segment fields as a structured array).  Returns per-episode
    (return, length, success, final contacts, per-step contact counts)."""
    E = int(sum(int(s["num_episodes"]) for s in segments))
    ret = np.zeros(E)
    length = np.zeros(E, np.int32)
    succ = np.zeros(E, bool)
    cont = np.zeros(E, np.int32)
    hist = [None] * E
    for lane in range(len(lane_off) - 1):
        pcur = 0
        ptape = policy_tapes[lane]
        for si in range(lane_off[lane], lane_off[lane + 1]):
            sg = segments[si]
            env = OracleEnv(cur=curricula[int(sg["curriculum_row"])], dense=dense,
                            max_episode_steps=max_episode_steps)
            o_on, d_on = sg["obs_noise_std"] > 0.0, sg["dyn_noise_std"] > 0.0
            ncur = int(sg["noise_offset"])
            for ep in range(int(sg["num_episodes"])):
                rec = int(sg["first_episode"]) + ep
                env.reset(reset_tape[rec])
                if o_on:
                    ncur += 45  # wrapper reset: obs noise (values unused by obs-independent policies)
                total, te, h = 0.0, False, []
                for step in range(max_steps):
                    a = oracle_policy_action(kind, mean[lane] if mean is not None else None, sigma,
                                             ptape[pcur:pcur + D])
                    pcur += D
                    if d_on:
                        g = noise_tape[ncur:ncur + D]
                        ncur += D
                        a = oracle_noisy_action(a, [0.0 + float(sg["dyn_noise_std"]) * x for x in g])
                    _, r, te, tr = env.step(a)
                    if o_on:
                        ncur += 45
                    total += r
                    h.append(env.num_contacts)
                    if te or tr:
                        break
                ret[rec], length[rec], succ[rec], cont[rec], hist[rec] = total, len(h), te, h[-1], h
    return ret, length, succ, cont, hist


# ---------------------------------------------------------------- device RNG restatement
_PH_M0, _PH_M1, _PH_W0, _PH_W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_STREAM_RESET = 0x52535400  # csrc/dxrl_device.h kStreamReset
_U32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Salmon et al., SC'11; Random123): 10 rounds of the two 32x32->64
    multiplies, Weyl key bumps (csrc/dxrl_device.h philox)."""
    x, y, z, w = (int(v) & _U32 for v in ctr)
    k0, k1 = int(key[0]) & _U32, int(key[1]) & _U32
    for _ in range(10):
        p0, p1 = _PH_M0 * x, _PH_M1 * z
        x, y, z, w = ((p1 >> 32) ^ y ^ k0) & _U32, p1 & _U32, ((p0 >> 32) ^ w ^ k1) & _U32, p0 & _U32
        k0, k1 = (k0 + _PH_W0) & _U32, (k1 + _PH_W1) & _U32
    return x, y, z, w


def env_key(seed: int, gid: int):
    """Per-env Philox key from (VecEnv seed, global env id) (csrc/dxrl_device.h env_key)."""
    seed &= (1 << 64) - 1
    k0 = ((gid & _U32) ^ (((seed >> 32) * 0x85EBCA6B) & _U32)) & _U32
    k1 = ((seed & _U32) ^ ((((gid >> 32) & _U32) * 0xC2B2AE35) & _U32)) & _U32
    return k0, k1


def _u01_53(hi, lo):
    return float(((hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0)


def philox_reset_draws(cur: OracleCurriculum, k0: int, k1: int, ctr: int) -> np.ndarray:
    """The 21 reset slots of a device-RNG reset with counter ``ctr`` (csrc/dxrl_device.h
    env_reset_philox): slot k is the 53-bit uniform of Philox block k // 2 (half k % 2);
    jp = -0.1 + 0.2 u, size / mass / friction / spawn = lo + (hi - lo) u (the reference's
    uniform(low, high) form, experiments/config.py:44-113); NaN where the curriculum has no
    range (the constant is used)."""
    u = []
    for b in range((D + 6 + 1) // 2):
        r = philox4x32_10((ctr & _U32, (ctr >> 32) & _U32, _STREAM_RESET, b), (k0, k1))
        u += [_u01_53(r[0], r[1]), _u01_53(r[2], r[3])]
    d = np.empty(D + 6)
    for k in range(D):
        d[k] = -0.1 + (0.1 - -0.1) * u[k]
    rngs = (cur.size_range, cur.mass_range, cur.friction_range, cur.spawn_x_range, cur.spawn_y_range,
            cur.spawn_z_range)
    for k, rg in enumerate(rngs):
        d[D + k] = math.nan if rg is None else rg[0] + (rg[1] - rg[0]) * u[D + k]
    return d


# ---------------------------------------------------------------- device noise streams (config C5)
STREAM_POLICY, STREAM_DYN, STREAM_OBS = 0x504F4C00, 0x44594E00, 0x4F425300  # csrc/dxrl_device.h kStream*


_P2_M, _P2_W = 0xD256D193, 0x9E3779B9


def philox2x32_10(ctr, key):
    """Philox2x32-10 (Salmon et al., SC'11; Random123): 10 rounds of the 32x32->64 multiply by
    0xD256D193 with a Weyl key bump (csrc/dxrl_device.h philox2x32_10)."""
    x, y = (int(v) & _U32 for v in ctr)
    k = int(key) & _U32
    for _ in range(10):
        p = _P2_M * x
        x, y = ((p >> 32) ^ k ^ y) & _U32, p & _U32
        k = (k + _P2_W) & _U32
    return x, y


def philox2x32_10_np(c0, c1, k, mid_round: int = -1):
    """Vectorised philox2x32_10 over NumPy arrays (uint64 lanes holding u32 values).  With
    ``mid_round`` r >= 0 also returns the first word after round r + 1 (the device's ``mid``)."""
    m = np.uint64(_U32)
    x, y = (np.asarray(v, np.uint64) & m for v in (c0, c1))
    k = np.asarray(k, np.uint64) & m
    mid = None
    for r in range(10):
        p = np.uint64(_P2_M) * x
        x, y = ((p >> np.uint64(32)) ^ k ^ y) & m, p & m
        k = (k + np.uint64(_P2_W)) & m
        if r == mid_round:
            mid = x
    return (x, y) if mid_round < 0 else (x, y, mid)


def device_normals_f64(key, ctr, stream: int, blocks: int) -> np.ndarray:
    """The device's fused-noise normals (csrc/dxrl_device.h noise_normals4: block b gives
    normals 4b .. 4b+3), restated in f64 with libm: Philox2x32-10 of (lo ctr, hi ctr << 8 ^
    stream ^ b) under k0 ^ k1 * 0x9E3779B9 -> (w0, w1), s = the first word after round 5;
    Box-Muller (r cos, r sin) of w0, then of w1, each with the angle u2 = (high 16 bits + 1) 2^-16
    and the radius uniform u1 = (v24 + 1) 2^-24, v24 = (word & 0xFFFF) << 8 | byte j of s (j = 0
    for w0, 1 for w1).  The device evaluates them with hardware log / sqrt / sin / cos in f32, so
    the values agree to ~1e-6 relative, not bit for bit: the tests use this to pin WHICH draws
    (key, counter, stream, block) a kernel consumed.  ``ctr``: uint64 array; ``key``: (k0, k1)
    arrays broadcastable to it.  Returns f64 [..., 4 * blocks]."""
    ctr = np.asarray(ctr, np.uint64)
    m = np.uint64(_U32)
    out = []
    for b in range(blocks):
        k = (np.asarray(key[0], np.uint64) ^ ((np.asarray(key[1], np.uint64) * np.uint64(_P2_W)) & m)) & m
        c1 = (((ctr >> np.uint64(32)) << np.uint64(8)) ^ np.uint64(stream) ^ np.uint64(b)) & m
        w0, w1, s = philox2x32_10_np(ctr & m, c1, np.broadcast_to(k, ctr.shape), mid_round=4)
        for j, w in enumerate((w0, w1)):
            e = (s >> np.uint64(8 * j)) & np.uint64(0xFF)
            v24 = ((w & np.uint64(0xFFFF)) << np.uint64(8)) | e
            ua = (v24.astype(np.float64) + 1.0) / 16777216.0
            ub = ((w >> np.uint64(16)).astype(np.float64) + 1.0) / 65536.0
            r = np.sqrt(-2.0 * np.log(ua))
            ang = 6.283185307179586 * ub
            out += [r * np.cos(ang), r * np.sin(ang)]
    return np.stack(out, axis=-1)
