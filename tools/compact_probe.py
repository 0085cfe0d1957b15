"""configs[4] (64 Ki fragmented messages) unmask variants, one batch in flight, for a kernel trace:
    rocprofv3 --kernel-trace --stats -d DIR -- python3 tools/compact_probe.py [iters]
Each variant decodes the same device batch `iters` times on one stream:
  c4  COMPACT, cache policy bits (unmask_nt >> 2) = 2 / 3 (loads nt bit 0, stores nt bit 1), windows
      of 4 and 8 KiB (WSC_UNMASK_CNT is passed through for A/B builds)
  c4i the same batch unmasked in place (the rate COMPACT is measured against)
and prints hipEvent ms per decode.  WSC_AB_NO_U8=1 in the environment runs the binary unmask."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from netman_amd import codec as K  # noqa: E402
from netman_amd import synth  # noqa: E402


def run(cfg, compact, nt, window, iters, cnt=0):
    os.environ["WSC_UNMASK_CNT"] = str(cnt)
    dev = torch.device("cuda:0")
    n = len(cfg["seg_off"]) - 1
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16,
                unmask_nt=nt, unmask_window=window)
    t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev), seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
             st=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), so=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
             fr=torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev), sm=torch.zeros(32, dtype=torch.uint8, device=dev))
    if compact:
        t["arena"] = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev)
        t["fd"] = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev)
    b = c.make_batch(t["wire"], t["seg_off"], None, t["st"], t["so"], t["fr"], t["sm"], compact=compact,
                     arena=t.get("arena"), frame_dst=t.get("fd"))
    st = torch.cuda.Stream(device=dev)
    for _ in range(3):
        c.decode(b, st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(iters):
        c.decode(b, st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"{'COMPACT' if compact else 'in place'} nt={nt:#x} window={window} cnt={cnt}: {ms:.4f} ms per decode, "
          f"errors {c.error_flags()}", flush=True)
    c.close()
    return t["arena"][:cfg["payload_bytes"] + 64].clone() if compact else None


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg = synth.fragmented_batch()
    print(f"configs[4]: {cfg['n_frames']} frames, {cfg['payload_bytes']} payload bytes, wire {len(cfg['wire'])}")
    ref = None
    variants = [(False, 3 | 2 << 2, 4096, 0), (True, 3 | 2 << 2, 4096, 0), (True, 3 | 3 << 2, 4096, 0),
                (True, 3 | 2 << 2, 8192, 0), (True, 3 | 0 << 2, 4096, 0), (True, 3 | 1 << 2, 4096, 0)]
    if os.environ.get("WSC_PROBE_VARIANT"):   # one variant alone (a PMC pass per variant)
        variants = [variants[int(os.environ["WSC_PROBE_VARIANT"])]]
    for compact, nt, window, cnt in variants:
        a = run(cfg, compact, nt, window, iters, cnt)
        if a is not None:   # every COMPACT variant writes the same arena
            ref = a if ref is None else ref
            print("  arena equal to the first COMPACT variant's:", bool(torch.equal(a, ref)), flush=True)


if __name__ == "__main__":
    main()
