"""Where does the header walk spend its time?  Per-block s_memrealtime stamps (wsc_config.walk_flags
WSC_WALK_DEBUG_STAMPS) for a workload; prints count / look-back / emit phase durations.
    python tools/walk_stamps.py <64k|1k|1k1|mixed|mixed1|frag> [walk_mode] [--lib path/to/libwscodec.so]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from netman_amd import codec as K, synth

args = sys.argv[1:]
if "--lib" in args:   # an A/B variant build (tools/build_variant.sh)
    i = args.index("--lib")
    K.load_library(os.path.abspath(args[i + 1]))
    del args[i:i + 2]
wl = args[0] if args else "64k"
mode = int(args[1]) if len(args) > 1 else 0
cfg = {"64k": lambda: synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1),
       "1k": lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1),
       "1k1": lambda: synth.uniform_batch(1 << 20, 1024, 1, seed=synth.SEED_BASE + 1),
       "mixed": lambda: synth.mixed_batch(),
       "mixed1": lambda: synth.mixed_batch(frames_per_seg=1),
       "frag": lambda: synth.fragmented_batch()}[wl]()
compact = wl == "frag"
dev = torch.device("cuda:0")
n = len(cfg["seg_off"]) - 1
c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16,
            walk_mode=mode, walk_flags=K.WALK_DEBUG_STAMPS)
t = [torch.from_numpy(cfg["wire"]).to(dev), torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
     torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), torch.zeros(n * 32, dtype=torch.uint8, device=dev),
     torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), torch.zeros(32, dtype=torch.uint8, device=dev)]
arena = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev) if compact else None
fdst = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev) if compact else None
b = c.make_batch(t[0], t[1], None, t[2], t[3], t[4], t[5], compact=compact, arena=arena, frame_dst=fdst)
n_cu = torch.cuda.get_device_properties(0).multi_processor_count
if mode == 0:
    mode = 65 if n <= 64 * n_cu else (256 if n <= 256 * n_cu else 3)
if mode == 3:   # the tiled walk (wsc_api.cpp): a persistent grid of 2 blocks per CU; stamps: start,
    # phase 1 counted, look-back done, phase 2 emitted
    nb = max(1, min(2 * n_cu, (n + 255) // 256))
    per = ((n + nb - 1) // nb + 255) // 256 * 256
    nb = (n + per - 1) // per
else:
    nb = (n + 63) // 64 if mode in (64, 65) else (n + 255) // 256
for it in range(3):
    c.decode(b)
    c.sync()
    out = np.zeros(nb * 8, np.uint64)
    assert c.lib.wsc_debug_stamps(c.h, out.ctypes.data, nb) == 0
    st = out.reshape(nb, 8).astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) / 100.0   # us
    if st[:, 4].min() > 0:
        pre = rel[:, 4] - rel[:, 0]
        print(f"{wl} iter {it}: quad pre-pass med {np.median(pre):.1f} max {pre.max():.1f} us")
    cnt = rel[:, 1] - rel[:, 0]
    lb = rel[:, 2] - rel[:, 1]
    em = rel[:, 3] - rel[:, 2]
    print(f"{wl} iter {it}: blocks={nb} start spread {rel[:,0].max():.1f} us | count med {np.median(cnt):.1f} max {cnt.max():.1f} | "
          f"lookback med {np.median(lb):.1f} max {lb.max():.1f} | emit med {np.median(em):.1f} max {em.max():.1f} | end {rel[:,3].max():.1f} us")
print(c.profile(b, 5))
