"""Interleaved A/B of one TrainerConfig knob in one process (same box, same clocks): two trainers
of workload CONFIG (default easy) with KNOB = A / B, whole PG iterations timed with HIP events in
alternating rounds after a shared prewarm.
usage: KNOB=fused_gnorm A=1 B=0 [CONFIG=easy EPOCHS=1 MINIBATCHES=1 ROUNDS=5 ITERS=20] python tools/knob_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.trainer import TrainerConfig  # noqa: E402
from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402


def parse(v):
    for f in (int, float):
        try:
            return f(v)
        except ValueError:
            pass
    return {"true": True, "false": False}.get(v.lower(), v)


knob = os.environ["KNOB"]
vals = {"A": parse(os.environ["A"]), "B": parse(os.environ["B"])}
if isinstance(getattr(TrainerConfig(), knob), bool):
    vals = {k: bool(v) for k, v in vals.items()}
cfg = os.environ.get("CONFIG", "easy")
ep, mb = int(os.environ.get("EPOCHS", "1")), int(os.environ.get("MINIBATCHES", "1"))
rounds, iters = int(os.environ.get("ROUNDS", "5")), int(os.environ.get("ITERS", "20"))
dev = torch.device("cuda:0")
trs = {k: build_pg_workload(cfg, dev, epochs=ep, minibatches=mb, **{knob: v})[1] for k, v in vals.items()}
t0 = time.time()
while time.time() - t0 < 2.0:  # clock prewarm, both trainers
    for tr in trs.values():
        tr.iteration()
torch.cuda.synchronize()
for r in range(rounds):
    for k, tr in trs.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            tr.iteration()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / iters
        print(f"round {r} {knob}={vals[k]} {ms:.4f} ms {tr.n * tr.T / ms / 1e3:.1f} M env-steps/s", flush=True)
