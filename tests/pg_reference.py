"""Plain-PyTorch fp32 reference of the policy-gradient learner (test-only).

The reference repository has no network / GAE / policy gradient, so this
restatement pins the HIP learner instead ("parity unpinned vs the
reference").  `loss_and_grads(..., bf16=True)` rounds to bf16 at exactly the
points the HIP pipeline stores bf16 (obs, weights, hidden activations,
head gradients, hidden gradients); `bf16=False` is the exact fp32 math,
checked against autograd in the CPU tests.
"""
import math

import torch

OBS_IN, IN, H, HX, OUT, ACT = 45, 64, 256, 288, 32, 15
W1, W2, W3 = H * IN, H * HX, OUT * HX
OFF = {"W1a": 0, "W2a": W1, "W3a": W1 + W2, "logstd": W1 + W2 + W3}
OFF["W1c"] = OFF["logstd"] + 32
OFF["W2c"] = OFF["W1c"] + W1
OFF["W3c"] = OFF["W2c"] + W2
NPARAMS = OFF["W3c"] + W3
LOG2PI = math.log(2 * math.pi)


def unpack(params):
    p = params
    blk = lambda name, r, c: p[OFF[name]:OFF[name] + r * c].view(r, c)  # noqa: E731
    out = {}
    for net in "ac":
        out[f"W1{net}"] = blk(f"W1{net}", H, IN)
        out[f"W2{net}"] = blk(f"W2{net}", H, HX)
        out[f"W3{net}"] = blk(f"W3{net}", OUT, HX)
    out["logstd"] = p[OFF["logstd"]:OFF["logstd"] + ACT]
    return out


def _r(x, bf16):
    return x.to(torch.bfloat16).float() if bf16 else x


def mlp_forward(X, Wd, net, bf16):
    """X [R][64] (col 45 = 1). Returns H1, H2 (stored precision) and the f32 head [R][32]."""
    W1_, W2_, W3_ = (_r(Wd[f"W{k}{net}"], bf16) for k in (1, 2, 3))
    b2 = Wd[f"W2{net}"][:, H]  # biases from the f32 master
    b3 = Wd[f"W3{net}"][:, H]
    H1 = _r(torch.tanh(X @ W1_.T), bf16)
    H2 = _r(torch.tanh(H1 @ W2_[:, :H].T + b2), bf16)
    head = H2 @ W3_[:, :H].T + b3
    return H1, H2, head


def gae_uses_segmented_scan(T):
    """dxrl_pg_gae's kernel choice (csrc/dxrl_pg.hip): k_gae_lds (segmented scan) while the horizon's
    LDS staging fits 152 KiB, else k_gae (one sequential chain per env)."""
    pitch = (T + 7) // 8 * 8 + 4
    return 16 * (12 * pitch + 4 * T) <= 152 * 1024


def gae(rew, done, V, n, T, gamma, lam, scan=None):
    """rew/done [T*n], V [(T+1)*n] -> adv, ret [T*n] (f32, the kernel's formula order).
    scan (default: the kernel's choice for T): k_gae_lds's segmented wavefront scan -- the horizon
    padded to 8-step chunks, 16 segments of whole chunks per env composed into affine maps, a
    Hillis-Steele suffix scan over the segments, each segment rerun from its incoming value --
    restated op for op; else the one-chain sequential recurrence of k_gae."""
    if scan is None:
        scan = gae_uses_segmented_scan(T)
    if scan:
        return _gae_segmented(rew, done, V, n, T, gamma, lam)
    rew, done, V = rew.view(T, n), done.view(T, n).float(), V.view(T + 1, n)
    adv = torch.empty(T, n, dtype=rew.dtype, device=rew.device)
    next_adv = torch.zeros(n, dtype=rew.dtype, device=rew.device)
    next_v = V[T]
    g = torch.tensor(gamma, dtype=rew.dtype)
    lm = torch.tensor(lam, dtype=rew.dtype)
    for t in range(T - 1, -1, -1):
        nd = 1.0 - done[t]
        delta = rew[t] + g * next_v * nd - V[t]
        a = delta + g * lm * nd * next_adv
        adv[t] = a
        next_adv = a
        next_v = V[t]
    ret = adv + V[:T]
    return adv.reshape(-1), ret.reshape(-1)


def _gae_segmented(rew, done, V, n, T, gamma, lam):
    rew, done, V = rew.view(T, n), done.view(T, n).float(), V.view(T + 1, n)
    dt, dev = rew.dtype, rew.device
    g = torch.tensor(gamma, dtype=dt)
    gl = g * torch.tensor(lam, dtype=dt)
    T8 = (T + 7) // 8 * 8
    delta = torch.zeros(T8, n, dtype=dt, device=dev)
    c = torch.zeros(T8, n, dtype=dt, device=dev)
    delta[:T] = rew + g * V[1:] * (1.0 - done) - V[:T]
    c[:T] = torch.where(done > 0, torch.zeros((), dtype=dt, device=dev), gl.to(dev))
    nc, S = T8 // 8, 16
    seg = [(8 * (s * nc // S), 8 * ((s + 1) * nc // S)) for s in range(S)]
    D = [torch.zeros(n, dtype=dt, device=dev) for _ in range(S)]
    C = [torch.ones(n, dtype=dt, device=dev) for _ in range(S)]
    for s, (lo, hi) in enumerate(seg):  # each segment's affine map from A_in = 0
        for t in range(hi - 1, lo - 1, -1):
            D[s] = delta[t] + c[t] * D[s]
            C[s] = c[t] * C[s]
    off = 1
    while off < S:  # suffix scan, every lane reading its neighbour's value of the previous step
        D, C = ([D[s] + C[s] * D[s + off] if s + off < S else D[s] for s in range(S)],
                [C[s] * C[s + off] if s + off < S else C[s] for s in range(S)])
        off *= 2
    adv = torch.empty(T8, n, dtype=dt, device=dev)
    for s, (lo, hi) in enumerate(seg):
        a = D[s + 1] if s + 1 < S else torch.zeros(n, dtype=dt, device=dev)
        for t in range(hi - 1, lo - 1, -1):
            a = delta[t] + c[t] * a
            adv[t] = a
    adv = adv[:T]
    ret = adv + V[:T]
    return adv.reshape(-1), ret.reshape(-1)


def loss_and_grads(params, obs_rm, act, logp_old, rew, done, n, T, cfg, bf16=True, norm_stats=None, total=None,
                   world=1, scales=None):
    """Manual forward/backward of the PPO objective as the HIP pipeline computes it.
    Sharded use (as PGTrainer with world > 1): norm_stats(adv) -> (mean, std) computed
    across ranks, total = global sample count, world = number of ranks; or
    scales = (per-sample loss scale, per-rank entropy coefficient) as
    distributed.loss_scales returns them (what the trainer hands the kernels).
    Returns (grads [NPARAMS], info dict)."""
    M = n * T
    total = M if total is None else total
    inv_total, ent = (1.0 / total, cfg["ent_coef"] / world) if scales is None else scales
    Wd = unpack(params)
    dt = params.dtype
    X = obs_rm.to(dt)
    H1c, H2c, vhead = mlp_forward(X, Wd, "c", bf16)
    V = vhead[:, 0]
    adv, ret = gae(rew.to(dt), done, V, n, T, cfg["gamma"], cfg["lam"])
    if norm_stats is None:
        mean, std = adv.double().mean(), adv.double().std()
    else:
        mean, std = norm_stats(adv)
    A = ((adv.double() - mean) / (std + 1e-8)).to(dt)
    Xa = X[:M]
    H1a, H2a, muh = mlp_forward(Xa, Wd, "a", bf16)
    mu = muh[:, :ACT]
    ls = Wd["logstd"]
    a = act[:, :ACT]
    iv = torch.exp(-2.0 * ls)
    z = (a - mu) * torch.exp(-ls)
    lp = (-0.5 * z * z - ls - 0.5 * LOG2PI).sum(1)
    ratio = torch.exp(lp - logp_old)
    s1, s2 = ratio * A, torch.clamp(ratio, 1 - cfg["clip_eps"], 1 + cfg["clip_eps"]) * A
    rc = torch.clamp(ratio, 1 - cfg["clip_eps"], 1 + cfg["clip_eps"])
    gsel = torch.where((s1 <= s2) | (ratio == rc), -A * ratio, torch.zeros_like(A)) * inv_total
    d = a - mu
    dmu = gsel[:, None] * d * iv
    dls = (gsel[:, None] * (d * d * iv - 1.0)).sum(0) - ent
    dv = 2.0 * cfg["vf_coef"] * (V[:M] - ret) * inv_total
    grads = torch.zeros(NPARAMS, dtype=dt, device=params.device)
    G = unpack(grads)
    G["logstd"].copy_(dls)
    for net, dY, H1, H2 in (("a", dmu, H1a, H2a), ("c", dv[:, None], H1c[:M], H2c[:M])):
        k = dY.shape[1]
        dYr = _r(dY, bf16)
        W2_, W3_ = _r(Wd[f"W2{net}"], bf16), _r(Wd[f"W3{net}"], bf16)
        G[f"W3{net}"][:k, :H] = dYr.T @ H2
        G[f"W3{net}"][:k, H] = dYr.sum(0)
        dH2 = _r((dYr @ W3_[:k, :H]) * (1 - H2 * H2), bf16)
        G[f"W2{net}"][:, :H] = dH2.T @ H1
        G[f"W2{net}"][:, H] = dH2.sum(0)
        dH1 = _r((dH2 @ W2_[:, :H]) * (1 - H1 * H1), bf16)
        G[f"W1{net}"][:, :] = dH1.T @ Xa
    loss = (-torch.minimum(s1, s2)).mean() + cfg["vf_coef"] * ((V[:M] - ret) ** 2).mean() - cfg["ent_coef"] * (
        ls.sum() + 0.5 * ACT * (1 + LOG2PI))
    return grads, {"V": V, "adv": adv, "ret": ret, "mu": muh, "mean": mean, "std": std, "loss": loss,
                   "ratio": ratio}


def autograd_loss(params, obs_rm, act, logp_old, rew, done, n, T, cfg):
    """The same objective through torch autograd (fp64 OK); adv/ret/normalisation are constants."""
    M = n * T
    params = params.detach().clone().requires_grad_(True)
    Wd = unpack(params)
    X = obs_rm.to(params.dtype)
    with torch.no_grad():
        _, _, vh = mlp_forward(X, {k: v.detach() for k, v in Wd.items()}, "c", False)
        adv, ret = gae(rew.to(params.dtype), done, vh[:, 0], n, T, cfg["gamma"], cfg["lam"])
        A = (adv - adv.mean()) / (adv.std() + 1e-8)
    _, _, vh = mlp_forward(X, Wd, "c", False)
    V = vh[:M, 0]
    _, _, muh = mlp_forward(X[:M], Wd, "a", False)
    mu, ls = muh[:, :ACT], Wd["logstd"]
    a = act[:, :ACT].to(params.dtype)
    lp = (-0.5 * ((a - mu) * torch.exp(-ls)) ** 2 - ls - 0.5 * LOG2PI).sum(1)
    ratio = torch.exp(lp - logp_old.to(params.dtype))
    s1 = ratio * A
    s2 = torch.clamp(ratio, 1 - cfg["clip_eps"], 1 + cfg["clip_eps"]) * A
    loss = (-torch.minimum(s1, s2)).mean() + cfg["vf_coef"] * ((V - ret) ** 2).mean() - cfg["ent_coef"] * (
        ls.sum() + 0.5 * ACT * (1 + LOG2PI))
    loss.backward()
    return params.grad.detach()


def fp64_pin(got_grads, got_V, got_adv, params, obs_rm, act, logp_old, rew, done, n, T, cfg, g_bf16, info_bf16,
             factor=1.5, blocks=("W1a", "W2a", "W3a", "W1c", "W2c", "W3c")):
    """Pin the HIP learner to fp64 truth, not just to the bf16 restatement:
    the same objective on the same tapes in float64 with no bf16 rounding anywhere is the truth;
    for every gradient block and for V / adv the HIP result's distance to it must be at most
    `factor` x the bf16-emulating torch reference's distance (both carry the same bf16 storage
    points, so a kernel regression that adds error shows as a ratio above 1).  Returns the
    ratios {name: |hip - truth| / |bf16 ref - truth|}."""
    g64, info64 = loss_and_grads(params.double(), obs_rm, act, logp_old, rew, done, n, T, cfg, bf16=False)
    got_b, ref_b, tru_b = unpack(got_grads), unpack(g_bf16), unpack(g64)
    ratios = {}
    pairs = [(b, got_b[b].double(), ref_b[b].double(), tru_b[b]) for b in blocks]
    pairs += [("V", got_V.double(), info_bf16["V"].double(), info64["V"]),
              ("adv", got_adv.double(), info_bf16["adv"].double(), info64["adv"])]
    for name, got, ref, tru in pairs:
        e_hip, e_ref = (got - tru).norm().item(), (ref - tru).norm().item()
        ratios[name] = e_hip / max(e_ref, 1e-300)
        assert e_hip <= factor * e_ref, (name, e_hip, e_ref)
    return ratios
