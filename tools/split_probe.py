"""Probe: does running the header walk on its own CU-masked stream let it overlap the other
in-flight batch's unmask?  Headline workload (16,384 x 64 KiB), two contexts in flight.

Variants (ms per step, median of 5 timed runs of K steps):
  base          wsc_decode, context j on torch stream j (what bench.py times)
  split/all     wsc_decode_split, walk stream and unmask stream both on all CUs
  split/K/lay   walk stream on K CUs, unmask stream on the other 256-K (lay: low bits or spread)
  walkK/all     walk stream on K CUs, unmask stream on all CUs
After each variant every in-flight buffer is checked against the numpy restatement (an even or
odd number of in-place decodes leaves it masked or unmasked)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

STEPS = int(os.environ.get("SPLIT_STEPS", "40"))
dev = torch.device("cuda:0")
cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)
n_bytes, n_segs = len(cfg["wire"]), len(cfg["seg_off"]) - 1
P = 2
codecs, batches, keep, count = [], [], [], [0] * P
for j in range(P):
    c = K.Codec(0, max_batch_bytes=n_bytes + 4096, max_segs=n_segs, max_frames=16384 + 16)
    t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev), seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
             st_out=torch.zeros(n_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
             seg_out=torch.zeros(n_segs * 32, dtype=torch.uint8, device=dev),
             frames=torch.zeros((16384 + 16) * 32, dtype=torch.uint8, device=dev),
             summ=torch.zeros(32, dtype=torch.uint8, device=dev))
    codecs.append(c)
    keep.append(t)
    batches.append(c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"]))
torch.cuda.synchronize()
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
sample = 64 * (65536 + 14)
kk = int(np.searchsorted(cfg["payload_off"] + cfg["plen"], sample, side="right"))
end = int(cfg["payload_off"][kk - 1] + cfg["plen"][kk - 1])
ref = synth.unmask_reference(cfg["wire"][:sample], cfg["payload_off"][:kk], cfg["plen"][:kk], cfg["mask"][:kk])


def check():
    torch.cuda.synchronize()
    ok = True
    for j in range(P):
        h = keep[j]["wire"][:sample].cpu().numpy()
        want = ref if count[j] % 2 else cfg["wire"][:sample]
        ok = ok and bool(np.array_equal(h[:end], want[:end]))
    return ok


def mask_of(cus):
    return K.cu_mask(cus, n_cu)


tstreams = [torch.cuda.Stream(device=dev) for _ in range(P)]


def time_it(step):
    res = []
    for _ in range(6):
        for i in range(5):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(STEPS):
            step(i)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / STEPS * 1e3)
    return float(np.median(res[1:])), res


def base_step(i):
    j = i % P
    codecs[j].decode(batches[j], tstreams[j].cuda_stream)
    count[j] += 1


ONLY = os.environ.get("SPLIT_ONLY", "")


def variant(name, walk_mask, unmask_mask, n_unmask=1):
    if ONLY and name not in ONLY.split(","):
        return
    ws = codecs[0].stream_create(walk_mask)
    us = [codecs[0].stream_create(unmask_mask) for _ in range(n_unmask)]

    def step(i):
        j = i % P
        codecs[j].decode_split(batches[j], ws, us[j % n_unmask])
        count[j] += 1
    med, res = time_it(step)
    ok = check()
    codecs[0].stream_destroy(ws)
    for u in us:
        codecs[0].stream_destroy(u)
    print(f"{name:22s} ms/step {med:.4f}  -> {1024 / med * 1e3 / 1024:8.1f} GiB/s  ok={ok}  all {[round(x, 4) for x in res]}", flush=True)


med, res = time_it(base_step) if not ONLY else (float("nan"), [])
print(f"{'base':22s} ms/step {med:.4f}  -> {1024 / med * 1e3 / 1024:8.1f} GiB/s  ok={check()}  all {[round(x, 4) for x in res]}", flush=True)
variant("split/all", None, None)
variant("split2/all", None, None, 2)
allc = list(range(n_cu))
for k in (8, 16, 32, 64):
    low = list(range(k))
    rest = [i for i in allc if i not in set(low)]
    variant(f"split/{k}/low", mask_of(low), mask_of(rest))
    variant(f"split2/{k}/low", mask_of(low), mask_of(rest), 2)
    variant(f"walk{k}low/all", mask_of(low), None)
    variant(f"walk{k}low/all x2", mask_of(low), None, 2)
for c in codecs:
    c.close()
