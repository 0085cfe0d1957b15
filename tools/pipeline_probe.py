"""Probe how well consecutive headline batches overlap on one device (bench.py's in-flight pipeline).

Variants, interleaved over rounds: 1 batch in flight; D batches on torch streams; D batches on raw
HIP streams (hipStreamCreateWithFlags non-blocking); D batches on raw streams created with the
highest priority.  Prints ms per step for each.
"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

STEPS = int(os.environ.get("STEPS", "40"))
DEPTH = int(os.environ.get("DEPTH", "2"))
dev = torch.device("cuda:0")
cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)
n_bytes = len(cfg["wire"])
n_segs = len(cfg["seg_off"]) - 1
codecs, batches, keep = [], [], []
for j in range(DEPTH):
    c = K.Codec(0, max_batch_bytes=n_bytes + 4096, max_segs=n_segs, max_frames=16384 + 16)
    t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev),
             seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
             st_out=torch.zeros(n_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
             seg_out=torch.zeros(n_segs * 32, dtype=torch.uint8, device=dev),
             frames=torch.zeros((16384 + 16) * 32, dtype=torch.uint8, device=dev),
             summ=torch.zeros(32, dtype=torch.uint8, device=dev))
    codecs.append(c)
    keep.append(t)
    batches.append(c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"]))

hip = C.CDLL("libamdhip64.so")
lo, hi = C.c_int(0), C.c_int(0)
hip.hipDeviceGetStreamPriorityRange(C.byref(lo), C.byref(hi))


def raw_streams(prio):
    out = []
    for _ in range(DEPTH):
        s = C.c_void_p()
        rc = hip.hipStreamCreateWithPriority(C.byref(s), 1, prio)
        assert rc == 0, rc
        out.append(s.value)
    return out


variants = {
    "single": [torch.cuda.current_stream().cuda_stream],
    "torch": [torch.cuda.Stream(device=dev).cuda_stream for _ in range(DEPTH)],
    "raw": raw_streams(lo.value),
    "raw_hiprio": raw_streams(hi.value),
}


def run(streams, steps):
    d = len(streams)
    for i in range(steps):
        codecs[i % DEPTH].decode(batches[i % DEPTH], streams[i % d])


res = {k: [] for k in variants}
for r in range(4):
    for k, st in variants.items():
        run(st, 6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(st, STEPS)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / STEPS * 1e3)
print(f"priority range {lo.value}..{hi.value}, depth {DEPTH}")
for k, v in res.items():
    print(f"{k:<12} ms/step median {np.median(v):.4f}  all {[round(x, 4) for x in v]}  "
          f"-> {cfg['payload_bytes'] / (np.median(v) * 1e-3) / 2**30:.1f} GiB/s")
for c in codecs:
    c.close()
