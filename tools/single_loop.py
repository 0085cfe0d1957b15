"""Back-to-back decodes of one device batch on one stream (one batch in flight), for kernel-trace
gap analysis:  python tools/single_loop.py <config> [iters] [--lib libwscodec.so]
config: head (16384 x 64 KiB, 4/seg) | c1 (1M x 1 KiB, 16/seg) | c2 (256k mixed, 16/seg) |
c4 (64k fragmented messages, COMPACT) | c4i (the same batch unmasked in place) |
t64 / t1 (TEXT 16384 x 64 KiB / 262144 x 1 KiB; wire restored before each decode, wall time includes the copy)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402


def main():
    args = sys.argv[1:]
    if "--lib" in args:   # an A/B build (tools/build_variant.sh) instead of the in-tree library
        i = args.index("--lib")
        K.load_library(os.path.abspath(args[i + 1]))
        del args[i:i + 2]
    which = args[0] if len(args) > 0 else "c1"
    iters = int(args[1]) if len(args) > 1 else 30
    cfg = {"head": lambda: synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1),
           "c1": lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1),
           "c11": lambda: synth.uniform_batch(1 << 20, 1024, 1, seed=synth.SEED_BASE + 1),
           "c2": lambda: synth.mixed_batch(),
           "c21": lambda: synth.mixed_batch(frames_per_seg=1),
           "c4": lambda: synth.fragmented_batch(),
           "c4i": lambda: synth.fragmented_batch(),
           "t64": lambda: synth.text_batch(16384, 65536, 4, seed=synth.SEED_BASE + 7),
           "t1": lambda: synth.text_batch(262144, 1024, 16, seed=synth.SEED_BASE + 8)}[which]()
    dev = torch.device("cuda:0")
    n = len(cfg["seg_off"]) - 1
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
    t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev), seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
             st=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), so=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
             fr=torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), sm=torch.zeros(32, dtype=torch.uint8, device=dev))
    compact = which == "c4"
    if compact:
        t["arena"] = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev)
        t["fd"] = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev)
    b = c.make_batch(t["wire"], t["seg_off"], None, t["st"], t["so"], t["fr"], t["sm"], compact=compact,
                     arena=t.get("arena"), frame_dst=t.get("fd"))
    st = torch.cuda.Stream(device=dev)
    # TEXT batches are decoded from the pristine masked wire every time (an in-place decode leaves
    # the payload unmasked; decoding it again would validate garbage); the copy is its own kernel
    pristine = t["wire"].clone() if which.startswith("t") else None

    def one():
        if pristine is not None:
            with torch.cuda.stream(st):
                t["wire"].copy_(pristine)
        c.decode(b, st.cuda_stream)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        one()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / iters * 1e3
    print(f"{which}: {el:.4f} ms per decode, {cfg['payload_bytes'] / (el * 1e-3) / 2**30:.1f} GiB/s, errors {c.error_flags()}")
    c.close()


if __name__ == "__main__":
    main()
