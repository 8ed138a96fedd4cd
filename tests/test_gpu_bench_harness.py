"""GPU: bench.py's own multi-rank harness, end to end.

`bench.py --gpus 2 --backend gloo` runs the path the driver's scaling runs take --
launch_ranks -> the torch.distributed.run child -> dist_setup at world 2 -> the trainer's
exchanges -> barrier -> max_over_ranks -> the rank-0 JSON line -- with both ranks on the one GPU
of a test box (gloo stages the exchanges through the host; RCCL needs a GPU per rank).  It is a
check of the harness, not a scaling measurement.  The reference has no multi-GPU path
(/root/reference/README.md:244-246)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config", ["easy", "default"])
def test_bench_two_ranks_over_gloo(config):
    envs, horizon, steps = 1024, 64, 3
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--config", config,
           "--envs", str(envs), "--horizon", str(horizon), "--steps", str(steps), "--warmup", "1",
           "--prewarm-s", "0.2", "--no-roofline", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps
    c = d["config"]
    assert c["world_size"] == 2 and c["envs_per_gpu"] == envs and c["global_envs"] == 2 * envs
    assert c["backend"].startswith("gloo") and c["ranks_per_gpu"] >= 1
    wall = d["ms_per_step"] * 1e-3 * steps
    want = 2 * envs * horizon * steps / wall
    assert abs(d["value"] - want) <= 1e-3 * want, (d["value"], want)
    # both shards trained: the episode statistics and losses are finite
    assert all(v == v for v in d["train_stats"].values() if isinstance(v, float))
