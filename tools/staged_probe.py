"""Staged split pipeline for one config with a chosen walk CU count and unmask CU mask (all CUs,
or only the CUs the walk does not use): per-batch wall time of two batches in flight.
    python tools/staged_probe.py <cfg> <walk_cus> <rest 0|1> [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402


def main():
    which, wcus, rest = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    cfg = {"head": lambda: synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1),
           "c1": lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1),
           "c2": lambda: synth.mixed_batch(),
           "c3": lambda: synth.uniform_batch(1 << 20, 4096, 16, seed=synth.SEED_BASE + 3),
           "t64": lambda: synth.text_batch(16384, 65536, 4, seed=synth.SEED_BASE + 7)}[which]()
    dev = torch.device("cuda:0")
    n = len(cfg["seg_off"]) - 1
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    pair = []
    for _ in range(2):
        c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
        t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev), seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
                 st=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), so=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
                 fr=torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), sm=torch.zeros(32, dtype=torch.uint8, device=dev))
        pair.append((c, c.make_batch(t["wire"], t["seg_off"], None, t["st"], t["so"], t["fr"], t["sm"]), t))
    torch.cuda.synchronize()
    c0 = pair[0][0]
    # PATTERN=stride: the walk's CUs are spread over the CU index space (i % 8 < wcus * 8 / n_cu)
    # instead of the first wcus indices (A/B for the XCD layout of the CU mask)
    if os.environ.get("PATTERN") == "stride":
        k8 = max(1, wcus * 8 // n_cu)
        wl = [i for i in range(n_cu) if i % 8 < k8]
    else:
        wl = list(range(wcus))
    rl = [i for i in range(n_cu) if i not in set(wl)]
    ws = c0.stream_create(K.cu_mask(wl, n_cu))
    us = c0.stream_create(K.cu_mask(rl, n_cu) if rest else None)

    def run(k):
        for i in range(k):
            cx, bx, _ = pair[i % 2]
            cx.decode_walk(bx, ws)
            cx.walk_wait()
            cx.decode_finish(bx, us)

    run(5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    ok = all(p[0].error_flags() == 0 for p in pair)
    print(f"{which} walk_cus {wcus} rest {rest}: {ms:.4f} ms per batch, {cfg['payload_bytes'] / (ms * 1e-3) / 2**30:.1f} GiB/s, ok {ok}")
    torch.cuda.synchronize()
    c0.stream_destroy(ws)
    c0.stream_destroy(us)


if __name__ == "__main__":
    main()
