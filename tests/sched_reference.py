"""NumPy restatement of dxrl_sched_scan (csrc/dxrl_sched.hip), test-only.

The rule it summarises is the reference's per-episode CurriculumScheduler feed
(experiments/curriculum_scheduler.py:116-170): the tests check this restatement
against one update() call per episode, and the kernel against this restatement."""
import numpy as np


def order_codes(codes):
    """u16 codes [world][T][N] -> the episode codes in (end step, global env id) order."""
    c = np.asarray(codes).astype(np.int64)
    seq = c.transpose(1, 0, 2).ravel()
    return seq[seq != 0]


def scan(codes, window, threshold, min_episodes, episodes_before, max_candidates, tail_codes):
    ep = order_codes(codes)
    tail = np.asarray(tail_codes, dtype=np.int64)
    succ, lens = ep & 1, ep >> 1
    tl, E = tail.size, ep.size
    cs = np.concatenate([[0], np.cumsum(np.concatenate([tail & 1, succ]))])
    k = np.arange(E)
    e = tl + k + 1
    win = cs[e] - cs[np.maximum(e - window, 0)]
    total = episodes_before + k + 1
    ok = (total >= min_episodes) & (total >= window) & (win / window >= threshold)
    csteps = np.cumsum(lens)
    cands = [(int(j), int(csteps[j]), int(win[j])) for j in np.nonzero(ok)[0][:max_candidates]]
    hist = np.concatenate([tail, ep])
    return {"episodes": E, "steps": int(lens.sum()), "successes": int(succ.sum()), "candidates": cands,
            "tail": hist[-window:] if hist.size else hist}
