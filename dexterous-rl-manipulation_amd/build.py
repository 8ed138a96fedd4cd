"""In-tree build of libdxrl.so for gfx950 (hipcc; no cmake, no JIT cache).

The built library lives next to this file so it travels with the repository
snapshot to the GPU box.  Numerics flags are part of the contract:
``-ffp-contract=off`` (the reference never fuses a multiply-add) and
correctly rounded f32 division/sqrt.
"""
from __future__ import annotations

import hashlib
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
SOURCES = ["dxrl_env.hip", "dxrl_rollout.hip", "dxrl_gemm.hip", "dxrl_pg.hip", "dxrl_pg_fused.hip", "dxrl_pg_rollout8.hip", "dxrl_eval.hip", "dxrl_sched.hip"]
HEADERS = ["dxrl_device.h", "dxrl_internal.h", "dxrl_mfma.h", "dxrl_gemm.h", "dxrl_pg.h", "dxrl_pg_rollout.h"]
OUT = os.path.join(PKG_DIR, "libdxrl.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -fno-slp-vectorize: no auto-packed f32 VALU (v_pk_*_f32), which costs extra issue cycles beside
# MFMAs on gfx950 (measured: -1.8 % per PG iteration, bit-identical results)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "-Wall", "-Wno-unused-function"]


def _inputs():
    root = os.path.dirname(PKG_DIR)
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    files.append(os.path.join(root, "include", "dxrl.h"))
    files.append(os.path.abspath(__file__))  # a flag change here must rebuild the library
    return files


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(f) <= t for f in _inputs())


ASAN_OUT = os.path.join(PKG_DIR, "libdxrl_asan.so")
# host-side AddressSanitizer on the C-ABI shim (argument checks, handle / layout logic, error
# plumbing); device code is compiled without it (GPU ASan is not available on this pool).  Load
# with LD_PRELOAD=asan_runtime() and DXRL_LIB=ASAN_OUT (tests/test_native_abi.py does).
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]


def asan_runtime() -> str:
    import glob
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else ""


def _jobs() -> int:
    try:
        return max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 1), 16))
    except ValueError:
        return 1


def build_native(force: bool = False, verbose: bool = False, asan: bool = False) -> str:
    """One object per translation unit (compiled in parallel, each rebuilt only when it or a
    header changed), then one link.  Every TU carries its own gfx950 code object (no -fgpu-rdc),
    as the single-command build did."""
    from concurrent.futures import ThreadPoolExecutor
    out = ASAN_OUT if asan else OUT
    if not force and os.path.exists(out) and all(os.path.getmtime(f) <= os.path.getmtime(out) for f in _inputs()):
        return out
    objdir = os.path.join(PKG_DIR, "_obj_asan" if asan else "_obj")
    os.makedirs(objdir, exist_ok=True)
    extra = ASAN_FLAGS if asan else []
    hdr_t = max(os.path.getmtime(f) for f in _inputs() if not f.endswith(".hip"))
    compile_flags = [f for f in FLAGS if f != "-shared"]

    def obj(src):
        o = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        s = os.path.join(CSRC, src)
        cmd = [HIPCC, *compile_flags, *extra, "-c", "-o", o + ".tmp", s]
        # the compile command's hash sits next to the object: a change of FLAGS, HIPCC or the
        # sanitizer options rebuilds it even when no source is newer
        stamp = o + ".cmd"
        digest = hashlib.sha256("\0".join(cmd).encode()).hexdigest()
        old = open(stamp).read().strip() if os.path.exists(stamp) else ""
        if (force or old != digest or not os.path.exists(o)
                or os.path.getmtime(o) < max(hdr_t, os.path.getmtime(s))):
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True, cwd=CSRC)
            os.replace(o + ".tmp", o)
            with open(stamp, "w") as f:
                f.write(digest + "\n")
        return o

    with ThreadPoolExecutor(_jobs()) as ex:
        objs = list(ex.map(obj, SOURCES))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *extra, "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
