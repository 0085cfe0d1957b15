"""A/B of the configs[0] echo decoders on one box: tools/ws_echo per-poller sessions (default),
--blocking-wait, --batcher (one batching thread per device), and the CPU port, at 1 / 4 / 8
pollers, 64 conns x 200 x 64 KiB and 64 conns x 2000 x 1 KiB, kinds interleaved, 3 reps each.
Prints one JSON line: {row: {kind: [GiB/s per rep]}}."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPU = os.path.join(ROOT, "tools", "ws_echo")
CPU = os.path.join(ROOT, "oracle", "_build", "ws_echo_cpu")
KINDS = {"gpu": (GPU, []), "gpu_blocking_wait": (GPU, ["--blocking-wait"]), "gpu_batcher": (GPU, ["--batcher"]),
         "gpu_batcher_bw": (GPU, ["--batcher", "--blocking-wait"]), "cpu_port": (CPU, [])}


def one(exe, args):
    p = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[-1]) if line else {}
    return d.get("gib_s") if d.get("ok") else None


res = {}
for P in (1, 4, 8):
    for size, frames in ((65536, 200), (1024, 2000)):
        row = f"64 conns x {frames} x {size} B, {P} poller(s)"
        args = ["--conns", "64", "--frames", str(frames), "--size", str(size), "--client-threads", "4", "--pollers", str(P)]
        got = {k: [] for k in KINDS}
        for _ in range(3):
            for k, (exe, extra) in KINDS.items():
                got[k].append(one(exe, args + extra))
        res[row] = got
        print(row, {k: v for k, v in got.items()}, flush=True)
print(json.dumps(res))
