"""Build an A/B variant of libdxrl.so into ab/lib<NAME>.so from the current csrc with text
substitutions applied to one source file (same flags as build.py).

    python tools/build_variant.py NAME [FILE OLD_TEXT_FILE NEW_TEXT_FILE ...]

With no substitutions the variant is the current tree.  Run A/B pairs on one box with
tools/ab.sh (DXRL_LIB selects the library)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dexterous-rl-manipulation_amd"))
import build as B  # noqa: E402

name, subs = sys.argv[1], sys.argv[2:]
out = os.path.join(ROOT, "ab", f"lib{name}.so")
os.makedirs(os.path.dirname(out), exist_ok=True)
# a mirror at the real depth keeps the sources' "../../include/dxrl.h" include working
src_root = os.path.join(ROOT, "ab", f"_src_{name}")  # per variant: builds may run in parallel
if os.path.exists(src_root):
    shutil.rmtree(src_root)
csrc = os.path.join(src_root, "pkg", "csrc")
rev = os.environ.get("SRC_REV")  # build the kernels of an older commit (same C ABI required)
if rev:
    os.makedirs(src_root)
    for sub, dst in (("dexterous-rl-manipulation_amd/csrc", csrc), ("include", os.path.join(src_root, "include"))):
        os.makedirs(dst)
        tar = subprocess.run(["git", "archive", rev, sub], cwd=ROOT, check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "--strip-components", str(sub.count("/") + 1), "-C", dst], input=tar, check=True)
else:
    shutil.copytree(B.CSRC, csrc)
    os.makedirs(os.path.join(src_root, "include"))
    shutil.copy(os.path.join(ROOT, "include", "dxrl.h"), os.path.join(src_root, "include", "dxrl.h"))
for k in range(0, len(subs), 3):
    fn, old, new = subs[k], open(subs[k + 1]).read(), open(subs[k + 2]).read()
    path = os.path.join(csrc, fn)
    txt = open(path).read()
    assert old in txt, f"{subs[k + 1]} not found in {fn}"
    open(path, "w").write(txt.replace(old, new))
subprocess.run([B.HIPCC, *B.FLAGS, *os.environ.get("EXTRA_FLAGS", "").split(), "-o", out, *[os.path.join(csrc, s) for s in B.SOURCES]], check=True, cwd=csrc)
shutil.rmtree(src_root)
print(out)
