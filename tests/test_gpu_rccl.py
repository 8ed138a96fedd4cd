"""GPU: the RCCL code path executed on the test box.  A one-GPU box cannot host two RCCL
ranks (RCCL wants one GPU per rank), so the worker joins a world-1 "nccl" process group
bound to cuda:0 (device_id) and runs, through distributed.py, every collective the sharded
trainer issues: the f32 SUM all-reduce of the gradient buffer, the all-gather of the f64
advantage-moment triple, the all-gather of the u16 episode codes as bytes, the int64
global_count SUM and the f64 MAX.  Each must return its input; and a PGTrainer driven
through that group (3 full iterations, curriculum-scheduler and fused-noise configs) must
give the group-less trainer's gradients, statistics, episode codes and parameters bit for
bit -- with its exchanges on the side stream overlapping the train passes (overlap_comm=True) and
serialised on the compute stream (overlap_comm=False, the default), with an iteration(update=False)
between updates (the overlapped form then issues no gradient collective and leaves none in
flight), and with CUs reserved for the collectives (reserve_cus).  Multi-rank semantics are covered by tests/test_dist_gloo.py (CPU) and
tests/test_gpu_dist.py (two ranks on one GPU over gloo)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_world1_collectives_and_trainer(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "rccl.pt")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py"), out], env=env, timeout=240)
    assert r.returncode == 0
    res = torch.load(out, weights_only=False)
    assert res["backend"] == "nccl"
    assert res["allreduce_equal"] and res["moments_equal"] and res["codes_equal"]
    assert res["global_count"] == 12345 and res["max"] == 3.25
    for config in ("default", "variable"):
        a, b, c = res[config]
        assert a["collective"] and not b["collective"] and c["collective"]
        assert a["overlapped"] and not c["overlapped"]
        for other in (b, c):
            for k in ("grads", "stats", "codes"):
                assert len(a[k]) == len(other[k])
                for x, y in zip(a[k], other[k]):
                    assert torch.equal(x, y), (config, k)
            assert torch.equal(a["params"], other["params"]), config
            if config == "default":
                assert a["sched"] == other["sched"]
        for suffix in ("_noupdate", "_reserve", "_paired"):
            a, b = res[config + suffix]
            assert a["collective"] and a["overlapped"] == (suffix != "_paired")
            for k in ("grads", "stats", "codes"):
                assert len(a[k]) == len(b[k])
                for x, y in zip(a[k], b[k]):
                    assert torch.equal(x, y), (config, suffix, k)
            assert torch.equal(a["params"], b["params"]), (config, suffix)
            if config == "default":
                assert a["sched"] == b["sched"]
