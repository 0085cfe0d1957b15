"""PCIe probe for the host-inclusive path: pinned H2D alone, D2H alone, and both at once on two
streams (does the link overlap the two directions for this process?).  Prints GB/s."""
import time

import torch

N = 256 << 20
dev = torch.device("cuda:0")
h_in = torch.empty(N, dtype=torch.uint8).pin_memory()
h_out = torch.empty(N, dtype=torch.uint8).pin_memory()
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.empty(N, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


def both_chunked(k=16):
    c = N // k
    for i in range(k):
        with torch.cuda.stream(s1):
            d_a[i * c:(i + 1) * c].copy_(h_in[i * c:(i + 1) * c], non_blocking=True)
        with torch.cuda.stream(s2):
            h_out[i * c:(i + 1) * c].copy_(d_b[i * c:(i + 1) * c], non_blocking=True)


t1, t2, t3, t4 = timed(h2d), timed(d2h), timed(both), timed(both_chunked)
print(f"H2D alone   {N / t1 / 1e9:6.1f} GB/s")
print(f"D2H alone   {N / t2 / 1e9:6.1f} GB/s")
print(f"both        {2 * N / t3 / 1e9:6.1f} GB/s aggregate ({t3 * 1e3:.2f} ms vs serial {(t1 + t2) * 1e3:.2f} ms)")
print(f"both 16x    {2 * N / t4 / 1e9:6.1f} GB/s aggregate ({t4 * 1e3:.2f} ms)")
