"""Time dxrl_gemm_bf16 / dxrl_wgrad_bf16 variants at the learner's shapes (HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dexterous_rl_manipulation_amd  # noqa: E402,F401
from dexterous_rl_manipulation_amd import _native as N  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("GM_M", str(819200)))
p = N.ptr
s = N.stream_of(dev)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


A = torch.randn(M, 288, device=dev).to(torch.bfloat16)
W = torch.randn(256, 288, device=dev).to(torch.bfloat16)
bias = torch.randn(256, device=dev)
gate = torch.randn(M, 288, device=dev).to(torch.bfloat16)
Crm = torch.empty(M, 288, device=dev, dtype=torch.bfloat16)
Cf = torch.empty(M, 256, device=dev)


def g(K, act=0, use_bias=False, use_gate=False, rm=True, f32=False):
    N.call("dxrl_gemm_bf16", 0, p(A), 288, p(W), 288, M, 256, K, p(bias) if use_bias else None, 1, act,
           p(gate) if use_gate else None, 288, p(Cf) if f32 else None, 256, p(Crm) if rm else None, 288, None, 0,
           None, 0, 1, None, s)


flop = lambda K: 2 * M * 256 * K / 1e12  # noqa: E731
for name, fn, K in [("K256 no-output", lambda: g(256, rm=False), 256), ("K256 rm", lambda: g(256), 256),
                    ("K256 rm+bias+tanh", lambda: g(256, act=1, use_bias=True), 256),
                    ("K256 rm+gate", lambda: g(256, use_gate=True), 256),
                    ("K64 rm+tanh", lambda: g(64, act=1), 64), ("K32 rm+gate", lambda: g(32, use_gate=True), 32),
                    ("K256 f32 out", lambda: g(256, rm=False, f32=True), 256)]:
    us = timeit(fn)
    print(f"{name:22s} {us:9.1f} us  {flop(K) / (us * 1e-6):7.1f} TF/s")

Y = torch.randn(M, 256, device=dev).to(torch.bfloat16)
X = torch.randn(M, 288, device=dev).to(torch.bfloat16)
out = torch.empty(256, 288, device=dev)
part = torch.empty(256, 256, 288, device=dev)
for splits in (32, 128, 256):
    us = timeit(lambda: N.call("dxrl_wgrad_bf16", 0, p(Y), 256, 256, p(X), 288, 288, M, splits, p(part), p(out), s))
    print(f"wgrad 256x288 splits={splits:3d} {us:9.1f} us  {2 * M * 256 * 288 / 1e12 / (us * 1e-6):7.1f} TF/s")
