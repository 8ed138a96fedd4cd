"""CPU checks of the C ABI: the library loads, exports every declared symbol,
and the ctypes mirrors have the C struct layouts (gcc-compiled probe)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dxrl.h")


@pytest.fixture(scope="module")
def native():
    import dexterous_rl_manipulation_amd as d
    from dexterous_rl_manipulation_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        d.build.build_native()
    return _native


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(dxrl_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    fns = declared_functions()
    assert "dxrl_env_step" in fns and "dxrl_rollout_simple" in fns and len(fns) >= 15


def test_library_exports_every_declared_symbol(native):
    lib = native.lib()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    assert set(declared_functions()) <= set(native._SIGS), "ctypes signatures missing"
    assert lib.dxrl_abi_version() == native.ABI_VERSION


def test_invalid_config_reports_error(native):
    cfg = native.EnvConfig()
    cfg.num_envs, cfg.num_fingers, cfg.joints_per_finger, cfg.reward_type = 8, 4, 3, 1
    lay = native.EnvLayout()
    with pytest.raises(ValueError, match="num_fingers"):
        native.call("dxrl_env_layout_for", C.byref(cfg), C.byref(lay))
    cfg.num_fingers, cfg.num_envs = 5, 0
    with pytest.raises(ValueError, match="num_envs"):
        native.call("dxrl_env_layout_for", C.byref(cfg), C.byref(lay))


def test_layout_is_aligned_and_sized(native):
    cfg = native.EnvConfig()
    cfg.num_envs, cfg.num_fingers, cfg.joints_per_finger, cfg.reward_type = 4099, 5, 3, 1
    lay = native.EnvLayout()
    native.call("dxrl_env_layout_for", C.byref(cfg), C.byref(lay))
    offs = [getattr(lay, f) for f, _ in native.EnvLayout._fields_[1:]]
    assert all(o % 256 == 0 for o in offs)
    assert offs == sorted(offs)
    assert lay.jv - lay.jp >= 4 * 15 * 4099 and lay.total_bytes > lay.curricula


def test_gae_partial_size_query(native):
    """dxrl_pg_gae's moment scratch: one (count, mean, M2) f64 triple per 16-env workgroup of
    k_gae_lds, the kernel with the most workgroups (include/dxrl.h)."""
    for n, T in ((1, 1), (16, 200), (17, 200), (8192, 32), (6000, 8), (65536, 1), (200, 800)):
        assert native.gae_partial_doubles(n, T) == 3 * ((n + 15) // 16)
    with pytest.raises(ValueError):
        native.gae_partial_doubles(0, 5)


def test_gnorm_partials_query_and_argument_checks(native):
    """dxrl_pg_gnorm_blocks: one f64 partial per block of the paired reduction (both networks'
    fused-pass slab blocks and dW2 blocks: 2 x (ceil(16,720 / 4 / 16) + 256 x 256 / 64) = 2,572);
    dxrl_pg_fused_pair_gnorm / dxrl_pg_adam_step reject bad arguments before touching a device."""
    nb = C.c_int32()
    native.call("dxrl_pg_gnorm_blocks", C.byref(nb))
    assert nb.value == 2 * ((16720 // 4 + 15) // 16 + 256 * 256 // 64) == 2572
    a, c = native.PgFusedArgs(), native.PgFusedArgs()
    with pytest.raises(ValueError, match="gnorm_blocks"):
        native.call("dxrl_pg_fused_pair_gnorm", 0, C.byref(c), C.byref(a), 4096, 2572, None, None)
    with pytest.raises(ValueError, match="2572 doubles"):  # checked before any launch
        native.call("dxrl_pg_fused_pair_gnorm", 0, C.byref(c), C.byref(a), 4096, 2571, C.byref(nb), None)
    fake = 1 << 20  # never dereferenced: the checks run first
    # a batch of one 32-row chunk: the dW2 split counts would be capped to 1, so the call must fail
    # before any launch (it failed only after overwriting dH2's partial slabs)
    for x, net in ((c, 1), (a, 0)):
        x.net, x.train, x.rows, x.grid, x.wgrad_splits, x.h1_mode = net, 1, 32, 256, 128, 0
        for k in ("packed", "params", "obs", "act", "logp_old", "adv", "ret", "stats", "loss_partial", "grads"):
            setattr(x, k, fake)
    c.dh2, a.dh2, c.partial, a.partial, c.wgrad_partial, a.wgrad_partial = (fake + 4096 * i for i in range(1, 7))
    with pytest.raises(ValueError, match="rows / 32"):
        native.call("dxrl_pg_fused_pair_gnorm", 0, C.byref(c), C.byref(a), 4096, 2572, C.byref(nb), None)
    c.rows = a.rows = 32 * 17
    with pytest.raises(ValueError, match="wgrad_splits"):
        c.wgrad_splits = 16
        native.call("dxrl_pg_fused_pair_gnorm", 0, C.byref(c), C.byref(a), 4096, 2572, C.byref(nb), None)
    # the stored layer-2 rows move in 16-byte pieces: misaligned pointers are refused up front
    c.rows = a.rows = 32 * 256
    c.wgrad_splits = 128
    a.h2_in = fake + 8
    with pytest.raises(ValueError, match="h2_in must be 16-byte aligned"):
        native.call("dxrl_pg_fused_pair_gnorm", 0, C.byref(c), C.byref(a), 4096, 2572, C.byref(nb), None)
    with pytest.raises(ValueError, match="h2_in / h2_out must be 16-byte aligned"):
        native.call("dxrl_pg_fused", 0, C.byref(a), None)
    a.h2_in = None
    with pytest.raises(ValueError, match="padded parameter count"):
        native.call("dxrl_pg_adam_step", 0, *([fake] * 7), 12345, 3e-4, 0.9, 0.999, 1e-5, 1, 0.5, fake, 2572, fake,
                    fake, None)
    with pytest.raises(ValueError, match="adam_step"):
        native.call("dxrl_pg_adam_step", 0, *([fake] * 7), 12345, 3e-4, 0.9, 0.999, 1e-5, 1, 0.5, fake, 0, fake,
                    fake, None)


STRUCTS = ["dxrl_curriculum", "dxrl_env_config", "dxrl_env_layout", "dxrl_learner_layout", "dxrl_learner_config",
           "dxrl_rollout_io", "dxrl_pg_rollout_args", "dxrl_pg_heads_args",
           "dxrl_pg_fused_args", "dxrl_eval_segment", "dxrl_eval_args", "dxrl_sched_args", "dxrl_sched_packed_args"]


def test_ctypes_struct_layouts_match_c(native):
    mirror = {"dxrl_curriculum": native.Curriculum, "dxrl_env_config": native.EnvConfig,
              "dxrl_env_layout": native.EnvLayout, "dxrl_learner_layout": native.LearnerLayout,
              "dxrl_learner_config": native.LearnerConfig, "dxrl_rollout_io": native.RolloutIO,
              "dxrl_pg_rollout_args": native.PgRolloutArgs, "dxrl_pg_heads_args": native.PgHeadsArgs,
              "dxrl_pg_fused_args": native.PgFusedArgs, "dxrl_eval_segment": native.EvalSegment,
              "dxrl_eval_args": native.EvalArgs, "dxrl_sched_args": native.SchedArgs,
              "dxrl_sched_packed_args": native.SchedPackedArgs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for s in STRUCTS:
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f, _ in mirror[s]._fields_:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "probe")
        subprocess.run(["gcc", "-std=c99", "-o", exe, c], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(line.split() for line in out if line)
    for s in STRUCTS:
        assert int(got[s]) == C.sizeof(mirror[s]), s
        for f, _ in mirror[s]._fields_:
            assert int(got[f"{s}.{f}"]) == getattr(mirror[s], f).offset, f"{s}.{f}"


def test_abi_checks_under_host_asan():
    """The C-ABI shim's host code (argument validation, layout queries, error strings, the
    struct-layout probe) under AddressSanitizer: this file's other tests re-run in a child
    process against libdxrl_asan.so (host code built with -fsanitize=address, __graft_entry__
    .build() builds it) with the clang ASan runtime preloaded.  Any ASan report fails the run."""
    import os
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "dexterous-rl-manipulation_amd"))
    import build as B
    rt = B.asan_runtime()
    if not rt or not os.path.exists(B.ASAN_OUT):
        pytest.skip("libdxrl_asan.so not built (run __graft_entry__.build())")
    env = dict(os.environ, LD_PRELOAD=rt, DXRL_LIB=B.ASAN_OUT, DXRL_ASAN_CHILD="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", os.path.abspath(__file__),
                        "-k", "not host_asan"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, r.stdout[-2000:] + r.stderr[-2000:]
