"""What does a stream dependency cost between two decodes on one stream?  50 back-to-back decodes
of the headline batch on one stream, plain / with an event record after each / with a wait on an
already-completed event before each / both (raw HIP events through the library's split API are
not involved: torch events, timing disabled).  Prints ms per decode for each variant."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from netman_amd import codec as K, synth

cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)
dev = torch.device("cuda:0")
n = len(cfg["seg_off"]) - 1
c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
t = [torch.from_numpy(cfg["wire"]).to(dev), torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
     torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), torch.zeros(n * 32, dtype=torch.uint8, device=dev),
     torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), torch.zeros(32, dtype=torch.uint8, device=dev)]
b = c.make_batch(t[0], t[1], None, t[2], t[3], t[4], t[5])
st = torch.cuda.Stream(device=dev)
other = torch.cuda.Stream(device=dev)
done = torch.cuda.Event()
done.record(other)
torch.cuda.synchronize()


def run(variant, reps=50):
    ev = [torch.cuda.Event() for _ in range(reps)]
    for i in range(5):
        c.decode(b, st.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        if variant in ("wait", "both"):
            st.wait_event(done)
        c.decode(b, st.cuda_stream)
        if variant in ("record", "both"):
            ev[i].record(st)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for v in ("plain", "record", "wait", "both", "plain"):
    print(f"{v:7s} {run(v):.4f} ms per decode", flush=True)
