"""Evaluation metrics -- evaluation/metrics.py:15-289, over episode arrays.

The reference classifies and aggregates a list of per-episode dicts one dict
at a time.  Here the core works on columns (success, steps, num_contacts,
final_contacts and the per-episode contact-count history moments that the
device evaluator produces); the reference's dict API is a thin adapter over
it.  Results are the reference's bit for bit:

* means / std go through the same NumPy reductions on the same int64 / f64
  arrays the reference builds from its lists;
* the variance rule ``np.var(counts) > 2.0`` (metrics.py:74-77) is decided
  exactly in integers, n*S2 - S1^2 > 2 n^2, and the rows where the true variance
  is exactly 2.0 are settled by np.var itself (its rounding decides them);
* the slippage rule (:80-83) is the same elementwise f64 expression
  (L / 5.0) - (F / 5.0) < -1.0 that np.mean produces for 5-element int lists.
"""
from __future__ import annotations

from enum import Enum
from typing import Dict, List, Optional, Sequence

import numpy as np


class FailureType(Enum):
    """metrics.py:15-22 (values are the reference's strings)."""
    SLIPPAGE = "slippage"
    UNSTABLE_CONTACTS = "unstable_contacts"
    MISALIGNED_GRASP = "misaligned_grasp"
    TIMEOUT = "timeout"
    OBJECT_DROPPED = "object_dropped"
    INSUFFICIENT_CONTACTS = "insufficient_contacts"


_TYPES = list(FailureType)  # code k <-> _TYPES[k]; -1 = success (no failure)
_CODE = {t: k for k, t in enumerate(_TYPES)}
_EXACT_VAR_MAX_N = 1 << 12  # integer variance test is exact far beyond this; beyond it defer to np.var


class HistoryMoments:
    """Per-episode contact-count history reduced to what the failure rules read:
    length n, S1 = sum c, S2 = sum c^2, F / L = sums of the first / last five
    counts, plus a row accessor for the rare exact-tie rows."""

    def __init__(self, n, s1, s2, first5, last5, row_fn):
        self.n = np.asarray(n, dtype=np.int64)
        self.s1 = np.asarray(s1, dtype=np.int64)
        self.s2 = np.asarray(s2, dtype=np.int64)
        self.first5 = np.asarray(first5, dtype=np.int64)
        self.last5 = np.asarray(last5, dtype=np.int64)
        self.row = row_fn

    @classmethod
    def from_lists(cls, histories: Sequence[Sequence[int]]) -> "HistoryMoments":
        rows = [np.asarray(h, dtype=np.int64) for h in histories]
        return cls([len(r) for r in rows], [int(r.sum()) for r in rows], [int((r * r).sum()) for r in rows],
                   [int(r[:5].sum()) for r in rows], [int(r[-5:].sum()) for r in rows], lambda i: rows[i])

    @classmethod
    def from_padded(cls, hist: np.ndarray, lengths: np.ndarray) -> "HistoryMoments":
        """hist u8 [E][max_steps] (device contact_hist), valid prefix lengths [E]."""
        h = hist.astype(np.int64)
        lengths = np.asarray(lengths, dtype=np.int64)
        steps = np.arange(h.shape[1])[None, :]
        valid = steps < lengths[:, None]
        hv = np.where(valid, h, 0)
        s1 = hv.sum(1)
        s2 = (hv * hv).sum(1)
        first5 = np.where(steps < np.minimum(lengths, 5)[:, None], h, 0).sum(1)
        last5 = np.where(valid & (steps >= (lengths - 5)[:, None]), h, 0).sum(1)
        return cls(lengths, s1, s2, first5, last5, lambda i: h[i, :lengths[i]])


def classify_columns(success, steps, num_contacts, final_contacts, moments: HistoryMoments, max_steps: int,
                     success_threshold: int = 3) -> np.ndarray:
    """Failure code per episode (-1 = success), metrics.py:39-103 in rule order."""
    success = np.asarray(success, dtype=bool)
    steps = np.asarray(steps, dtype=np.int64)
    nc = np.asarray(num_contacts, dtype=np.int64)
    fc = np.asarray(final_contacts, dtype=np.int64)
    n = moments.n
    code = np.full(success.shape, -1, dtype=np.int64)
    open_ = ~success

    def assign(mask, t):
        nonlocal open_
        m = open_ & mask
        code[m] = _CODE[t]
        open_ = open_ & ~m

    assign(steps >= max_steps, FailureType.TIMEOUT)          # :63-65
    assign(fc == 0, FailureType.OBJECT_DROPPED)              # :67-69
    # :72-83 -- only when the history has more than 5 entries
    num = n * moments.s2 - moments.s1 * moments.s1           # n^2 var, exact
    lim = 2 * n * n
    unstable = (n > 5) & (num > lim)
    tie = open_ & (n > 5) & ((num == lim) | (n > _EXACT_VAR_MAX_N))
    for i in np.flatnonzero(tie):
        unstable[i] = bool(np.var(moments.row(i)) > 2.0)
    assign(unstable, FailureType.UNSTABLE_CONTACTS)
    trend = (moments.last5.astype(np.float64) / 5.0) - (moments.first5.astype(np.float64) / 5.0)
    assign((n > 10) & (trend < -1.0), FailureType.SLIPPAGE)
    assign((nc > 0) & (nc < success_threshold), FailureType.MISALIGNED_GRASP)  # :86-87
    assign(np.ones_like(success), FailureType.INSUFFICIENT_CONTACTS)           # :90-95
    return code


def _mean_or_none(x):
    return float(np.mean(x)) if len(x) else None


def aggregate_columns(success, steps, num_contacts, codes) -> Dict:
    """metrics.py:128-206 compute_aggregate_metrics over columns."""
    total = len(success)
    if total == 0:
        return {}
    success = np.asarray(success, dtype=bool)
    steps = np.asarray(steps, dtype=np.int64)
    nc = np.asarray(num_contacts, dtype=np.int64)
    codes = np.asarray(codes, dtype=np.int64)
    counts = np.bincount(codes[codes >= 0], minlength=len(_TYPES))
    freq = {t.value: {"count": int(counts[k]), "frequency": float(int(counts[k]) / total)}
            for k, t in enumerate(_TYPES)}
    ok, bad = success, ~success
    return {
        "grasp_success_rate": float(np.mean(success)),
        "mean_episode_length": float(np.mean(steps)),
        "std_episode_length": float(np.std(steps)),
        "failure_type_frequency": freq,
        "total_episodes": total,
        "successful_episodes": int(ok.sum()),
        "failed_episodes": int(bad.sum()),
        "mean_contacts": float(np.mean(nc)),
        "mean_success_length": _mean_or_none(steps[ok]),
        "mean_success_contacts": _mean_or_none(nc[ok]),
        "mean_failure_length": _mean_or_none(steps[bad]),
        "mean_failure_contacts": _mean_or_none(nc[bad]),
    }


def _history_counts(h) -> List[int]:
    """contact_history rows are 5-element 0/1 lists (evaluator.py:148-149); the
    rule counts entries > 0.5 (metrics.py:73)."""
    return [sum(1 for c in row if c > 0.5) for row in h]


def _columns_of(episodes: Sequence[Dict]):
    success = [bool(e.get("success", False)) for e in episodes]
    steps = [e.get("episode_steps", 0) for e in episodes]
    nc = [e.get("num_contacts", 0) for e in episodes]
    fc = [e.get("final_contacts", e.get("num_contacts", 0)) for e in episodes]
    hist = HistoryMoments.from_lists([_history_counts(e.get("contact_history", [])) for e in episodes])
    return success, steps, nc, fc, hist


class EvaluationMetrics:
    """metrics.py:25-229 (dict API) over the column core above."""

    def __init__(self, success_threshold: int = 3):
        self.success_threshold = success_threshold

    def _codes(self, episodes, max_steps):
        s, st, nc, fc, h = _columns_of(episodes)
        return classify_columns(s, st, nc, fc, h, max_steps, self.success_threshold), s, st, nc

    def classify_failure(self, episode_data: Dict, max_steps: int = 200) -> Optional[FailureType]:
        code = int(self._codes([episode_data], max_steps)[0][0])
        return None if code < 0 else _TYPES[code]

    def compute_episode_metrics(self, episode_data: Dict, max_steps: int = 200) -> Dict:
        ft = self.classify_failure(episode_data, max_steps)
        return {"success": episode_data.get("success", False),
                "episode_length": episode_data.get("episode_steps", 0),
                "num_contacts": episode_data.get("num_contacts", 0),
                "failure_type": ft.value if ft else None}

    def compute_aggregate_metrics(self, all_episodes: List[Dict], max_steps: int = 200) -> Dict:
        if not all_episodes:
            return {}
        codes, s, st, nc = self._codes(all_episodes, max_steps)
        return aggregate_columns(s, st, nc, codes)

    def compute_per_object_metrics(self, per_object_results: Dict, max_steps: int = 200) -> Dict:
        return {k: self.compute_aggregate_metrics(v["episodes"], max_steps)
                for k, v in per_object_results.items() if v.get("episodes")}

    # column entry points (device evaluator records)
    def classify_records(self, success, steps, num_contacts, final_contacts, moments, max_steps: int) -> np.ndarray:
        return classify_columns(success, steps, num_contacts, final_contacts, moments, max_steps,
                                self.success_threshold)


def failure_names(codes: np.ndarray) -> List[Optional[str]]:
    return [None if c < 0 else _TYPES[c].value for c in codes]


def format_metrics_report(metrics: Dict) -> str:
    """metrics.py:232-289: the reference's plain-text report, line for line."""
    bar = "=" * 60
    rate = metrics.get("grasp_success_rate", 0.0)
    status = ("PASS (>= 70%)" if rate >= 0.70 else "MARGINAL (50-70%)" if rate >= 0.50 else "FAIL (< 50%)")
    out = [bar, "Evaluation Metrics Report", bar,
           "\nOverall Statistics:",
           f"  Total episodes: {metrics.get('total_episodes', 0)}",
           f"  Successful episodes: {metrics.get('successful_episodes', 0)}",
           f"  Failed episodes: {metrics.get('failed_episodes', 0)}",
           f"\nGrasp Success Rate: {rate:.1%}",
           f"  Status: {status}",
           f"\nMean Episode Length: {metrics.get('mean_episode_length', 0.0):.1f} ± "
           f"{metrics.get('std_episode_length', 0.0):.1f} steps"]
    for key, label in (("mean_success_length", "Success"), ("mean_failure_length", "Failure")):
        if metrics.get(key):
            out.append(f"  {label} episodes: {metrics[key]:.1f} steps")
    out.append("\nFailure Type Frequency:")
    ranked = sorted(metrics.get("failure_type_frequency", {}).items(), key=lambda kv: kv[1]["count"], reverse=True)
    out += [f"  {name}: {d['count']} ({d['frequency']:.1%})" for name, d in ranked if d["count"] > 0]
    out += ["\nContact Statistics:", f"  Mean contacts: {metrics.get('mean_contacts', 0.0):.2f}"]
    for key, label in (("mean_success_contacts", "Success"), ("mean_failure_contacts", "Failure")):
        if metrics.get(key):
            out.append(f"  {label} episodes: {metrics[key]:.2f} contacts")
    out.append(bar)
    return "\n".join(out)
