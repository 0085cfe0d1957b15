"""Decode one TEXT batch (16,384 x 64 KiB valid UTF-8, the bench's TEXT line) a few times and
nothing else, so per-kernel PMC counters of k_u8_check (rocprofv3 --pmc) are not mixed with other
workloads.  Prints the per-kernel hipEvent times."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

n_frames = int(os.environ.get("U8_FRAMES", "16384"))
size = int(os.environ.get("U8_SIZE", "65536"))
cfg = synth.text_batch(n_frames, size, 4, seed=synth.SEED_BASE + 7)
dev = torch.device("cuda:0")
n = len(cfg["seg_off"]) - 1
c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
t = [torch.from_numpy(cfg["wire"]).to(dev), torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
     torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), torch.zeros(n * 32, dtype=torch.uint8, device=dev),
     torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), torch.zeros(32, dtype=torch.uint8, device=dev)]
b = c.make_batch(t[0], t[1], None, t[2], t[3], t[4], t[5])
for _ in range(int(os.environ.get("U8_ITERS", "5"))):
    print(c.profile(b, 1))
c.close()
