"""A few encodes of bench.py's two encode batches (for rocprofv3 --pmc passes; no timing).
usage: python tools/enc_loop.py [iters]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
for nf, size, fps in [(16384, 65536, 4), (1 << 20, 1024, 16)]:
    cfg = synth.uniform_batch(nf, size, fps, seed=synth.SEED_BASE + 1)
    n = int(cfg["n_frames"])
    msgs = np.zeros(n, K.OUT_MSG_DTYPE)
    msgs["src_off"], msgs["len"], msgs["first_byte"] = cfg["payload_off"], cfg["plen"], 0x82
    pl = cfg["plen"].astype(np.int64)
    total = int((pl + np.where(pl <= 125, 2, np.where(pl <= 65535, 4, 10))).sum())
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1024, max_frames=n + 16)
    src = torch.from_numpy(cfg["wire"]).to(dev)
    d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).to(dev)
    d_out = torch.empty(total + 4096, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    for _ in range(iters):
        c.encode(d_msgs, n, src, len(cfg["wire"]), d_out, total + 4096, d_off, 0)
    torch.cuda.synchronize()
    assert int(d_off[-1].item()) == total, (int(d_off[-1].item()), total)
    c.close()
print("ok")
