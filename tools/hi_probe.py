"""A/B of the host-inclusive pipelined leg (bench.host_inclusive_pipelined): pieces x copy-stream
layout, on the headline batch (16 Ki x 64 KiB).  usage: python tools/hi_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)
n_bytes, n_segs = len(cfg["wire"]), len(cfg["seg_off"]) - 1
codecs = [K.Codec(0, max_batch_bytes=n_bytes + 4096, max_segs=n_segs, max_frames=16384 + 16) for _ in range(2)]
streams = [torch.cuda.Stream() for _ in range(2)]
runs = [(16, True, 3, 1, 0), (16, False, 3, 1, 0), (16, False, 3, 1, 1), (16, False, 3, 1, 2), (32, False, 4, 1, 2),
        (16, False, 4, 1, 1), (32, False, 4, 1, 1)]
for chunks, ds, nbuf, cs, kc in runs + runs[:4]:
    r = bench.host_inclusive_pipelined(torch, codecs, streams, cfg, K, chunks=chunks, iters=3, dir_streams=ds,
                                       nbuf=nbuf, copy_streams=cs, kcopy=kc)
    print(f"chunks {chunks:3d} dir_streams {int(ds)} nbuf {nbuf} copy_streams {cs} kcopy {kc}: {r['gib_s']:6.2f} GiB/s  "
          f"{r['ms_per_batch']:7.2f} ms  parity {r['parity_ok']}", flush=True)
print("sync", bench.host_inclusive(codecs[0], cfg, K), flush=True)
for c in codecs:
    c.close()
