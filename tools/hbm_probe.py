"""HBM ceilings on this box (torch kernels over 671 MB buffers): read-only, write-only, copy, axpy."""
import torch

dev = torch.device("cuda:0")
n = 640 * 1024 * 1024 // 4  # 671 MB of f32 per buffer (well past the 256 MB Infinity Cache)
a = torch.empty(n, dtype=torch.float32, device=dev).uniform_()
b = torch.empty_like(a)


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


nb = a.numel() * 4
for name, fn, byts in [("read (sum)", lambda: a.sum(), nb), ("write (fill)", lambda: b.fill_(1.0), nb),
                       ("copy", lambda: b.copy_(a), 2 * nb), ("axpy-like (b=a*2)", lambda: torch.mul(a, 2.0, out=b), 2 * nb)]:
    ms = t(fn)
    print(f"{name:20s} {ms:.3f} ms {byts / ms / 1e9:.2f} TB/s")
