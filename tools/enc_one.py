"""One encode case, for profiling the encode kernels alone (rocprofv3 --kernel-trace --stats,
--pmc): loads the given libwscodec.so and runs 30 back-to-back encodes of the 1M x 1 KiB BIN echo
batch (bench.py encode_configs' second case) or, with "64k", of its 16384 x 64 KiB batch.
    python tools/enc_one.py <lib.so> [1k|64k]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from netman_amd import codec as K, synth  # noqa: E402

if __name__ == "__main__":
    K.load_library(os.path.abspath(sys.argv[1]))
    big = len(sys.argv) > 2 and sys.argv[2] == "64k"
    cfg = synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1) if big else \
        synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1)
    n = int(cfg["n_frames"])
    msgs = np.zeros(n, K.OUT_MSG_DTYPE)
    msgs["src_off"], msgs["len"], msgs["first_byte"] = cfg["payload_off"], cfg["plen"], 0x82
    dev = torch.device("cuda:0")
    c = K.Codec(0, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1024, max_frames=n + 16)
    src = torch.from_numpy(cfg["wire"]).to(dev)
    d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).to(dev)
    cap = int(cfg["payload_bytes"]) + 16 * n
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        for _ in range(30):
            c.encode(d_msgs, n, src, len(cfg["wire"]), d_out, cap, d_off, st.cuda_stream)
    st.synchronize()
    print("total", int(d_off[-1].item()))
    c.close()
