"""Segment stamps of the train passes at the bench shape (config_easy, 4096 x 200, 1 x 1), with the
stored layer-2 rows (VARIANT=both) or recomputing them (VARIANT=none). Needs a library built with
-DDXRL_H2_STAMPS=1 and DXRL_FUSED_DIAG=8 (the kernel prints its mean cycles per segment to stderr)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dexterous_rl_manipulation_amd.workloads import build_pg_workload  # noqa: E402

v = os.environ.get("VARIANT", "both")
env, tr = build_pg_workload("easy", torch.device("cuda:0"), envs=4096, horizon=200, reuse_h2=v != "none")
for _ in range(int(os.environ.get("REPS", "3"))):
    tr.iteration()
    torch.cuda.synchronize()
print(v, "ok")
