"""Sweep unmask-kernel knobs (window bytes, waves per CU, non-temporal flags) on one device in ONE
process, interleaved rounds (guide §5.4 rule 24).  Prints a table of per-kernel device times."""
import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="64k", choices=["64k", "1k", "mixed", "4k", "frag"])
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--windows", default="4096,8192")
ap.add_argument("--wpc", default="8,16,32,4096")
ap.add_argument("--nt", default="0,1,2,3")
ap.add_argument("--minw", default="0")
a = ap.parse_args()

if a.workload == "64k":
    cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)
elif a.workload == "4k":
    cfg = synth.uniform_batch(262144, 4096, 16, seed=synth.SEED_BASE + 3)
elif a.workload == "1k":
    cfg = synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1)
elif a.workload == "frag":
    cfg = synth.fragmented_batch()
else:
    cfg = synth.mixed_batch()
compact = a.workload == "frag"
dev = torch.device("cuda:0")
n_segs = len(cfg["seg_off"]) - 1
wire = torch.from_numpy(cfg["wire"]).to(dev)
seg_off = torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev)
st_out = torch.zeros(n_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev)
seg_out = torch.zeros(n_segs * 32, dtype=torch.uint8, device=dev)
frames = torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev)
summ = torch.zeros(32, dtype=torch.uint8, device=dev)
arena = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev) if compact else None
fdst = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev) if compact else None
hdr = np.where(cfg["plen"] <= 125, 6, np.where(cfg["plen"] <= 65535, 8, 14))
alg = int((2 * cfg["plen"].astype(np.int64) + hdr + 32).sum())
combos = list(itertools.product([int(x) for x in a.windows.split(",")], [int(x) for x in a.wpc.split(",")],
                                [int(x) for x in a.nt.split(",")], [int(x) for x in a.minw.split(",")]))
codecs = {}
for w, wpc, nt, mw in combos:
    codecs[(w, wpc, nt, mw)] = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n_segs,
                                       max_frames=cfg["n_frames"] + 16, unmask_window=w,
                                       unmask_waves_per_cu=wpc, unmask_nt=(nt << 2) if compact else nt, unmask_minw=mw)
res = {c: [] for c in combos}
for r in range(a.rounds):
    for c in combos:
        cd = codecs[c]
        b = cd.make_batch(wire, seg_off, None, st_out, seg_out, frames, summ, compact=compact, arena=arena, frame_dst=fdst)
        p = cd.profile(b, a.iters)
        res[c].append(p)
rows = []
for c in combos:
    um = float(np.median([p["unmask"] for p in res[c]]))
    tot = float(np.median([p["total"] for p in res[c]]))
    rows.append((um, c, tot))
rows.sort()
print(f"workload={a.workload} payload={cfg['payload_bytes']} alg_bytes={alg}")
for um, c, tot in rows:
    print(f"window={c[0]:6d} wpc={c[1]:5d} nt={c[2]} minw={c[3]}  unmask {um*1e3:8.1f} us  {alg/um/1e6:8.1f} GB/s  "
          f"total {tot*1e3:8.1f} us  payload {cfg['payload_bytes']/tot/1e6/1.073741824:8.1f} GiB/s")
best = rows[0]
print(json.dumps({"workload": a.workload, "best": {"window": best[1][0], "wpc": best[1][1], "nt": best[1][2],
                                                   "minw": best[1][3], "unmask_us": best[0] * 1e3}}))
