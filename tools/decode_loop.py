"""Decode one workload `iters` times (device-resident, one context, default stream): the program
rocprofv3 --pmc / --kernel-trace passes run to measure the header walk and the unmask of the
non-headline BASELINE configs (profiles/pmc_traffic.json "walk" section).
usage: python tools/decode_loop.py {1k,1k1,mixed,mixed1,frag,64k} [iters] [--time]
--time: also report the wall-clock time per decode of back-to-back decodes on one stream (no
events between the stages), i.e. the single-batch device time including kernel boundaries."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from netman_amd import codec as K, synth

WORKLOADS = {"64k": lambda: synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1),
             "1k": lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1),
             "1k1": lambda: synth.uniform_batch(1 << 20, 1024, 1, seed=synth.SEED_BASE + 1),
             "mixed": lambda: synth.mixed_batch(),
             "mixed1": lambda: synth.mixed_batch(frames_per_seg=1),
             "frag": lambda: synth.fragmented_batch()}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "1k"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cfg = WORKLOADS[wl]()
    compact = wl == "frag"
    dev = torch.device("cuda:0")
    n = len(cfg["seg_off"]) - 1
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
    t = [torch.from_numpy(cfg["wire"]).to(dev), torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
         torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), torch.zeros(n * 32, dtype=torch.uint8, device=dev),
         torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), torch.zeros(32, dtype=torch.uint8, device=dev)]
    arena = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev) if compact else None
    fdst = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev) if compact else None
    b = c.make_batch(t[0], t[1], None, t[2], t[3], t[4], t[5], compact=compact, arena=arena, frame_dst=fdst)
    for _ in range(iters):
        c.decode(b)
    c.sync()
    assert c.error_flags() == 0
    if "--time" in sys.argv:
        import time
        for _ in range(5):
            c.decode(b)
        c.sync()
        reps = 200
        t0 = time.perf_counter()
        for _ in range(reps):
            c.decode(b)
        c.sync()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"{wl}: back-to-back decode {ms:.4f} ms/batch = {cfg['payload_bytes'] / (ms * 1e-3) / 2**30:.1f} GiB/s", flush=True)
    p = c.profile(b, 10)
    print(f"{wl}: frames={cfg['n_frames']} segs={n} payload={cfg['payload_bytes']} " +
          " ".join(f"{k}={v:.4f}ms" for k, v in p.items()), flush=True)
    c.close()


if __name__ == "__main__":
    main()
