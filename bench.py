"""Benchmark: GiB/s of masked WebSocket payload unmasked, device-resident, 64 KiB-frame batch.

One step = one full batched decode (libwscodec wsc_decode: header walk -> scan -> record emit ->
XOR unmask in place -> utf8 pass) of a device-resident batch of 16,384 masked 64 KiB BIN frames
(1 GiB of payload, 14-byte headers, 4 frames per connection segment) per GPU.  Multi-GPU: one
process per GPU (torchrun), each rank decodes its own independent shard (seed + rank) -- the path
shards by connection with no collective; torch.distributed is used only for the barrier and the
max-over-ranks time.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FRAMES = 16384
FRAME_BYTES = 65536
FRAMES_PER_SEG = 4
RECORD_BYTES = 32          # sizeof(wsc_frame)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# (walk CUs, unmask only on the other CUs) tried for each other_configs line's pipelined column
# (0, 0): the walk on a high-priority stream over all CUs, the unmask on a normal one over all CUs;
# (-1, 0): serial -- both contexts' walks and unmasks in order on one stream, for configs whose
# latency-bound walk loses more beside an unmask than it saves (configs[1], [3]: the walk then
# slows past the unmask it hides behind, profiles/r05/ab1_*.log)
PIPELINE_SPLITS = [(-1, 0), (0, 0), (16, 0), (32, 1), (64, 1), (80, 1), (96, 1), (112, 1), (128, 1), (128, 0)]
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--frame-bytes", type=int, default=FRAME_BYTES)
    ap.add_argument("--frames-per-seg", type=int, default=FRAMES_PER_SEG)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--pipeline", type=int, default=2,
                    help="batches in flight: each has its own context, wire buffer and HIP stream, so the "
                         "header walk of batch k+1 overlaps the unmask of batch k")
    ap.add_argument("--walk-cus", type=int, default=16,
                    help="split pipeline (wsc_decode_split): the header walk runs on a stream masked to this "
                         "many CUs, the unmask (+ UTF-8 check when text was deferred) on --unmask-streams streams over every CU "
                         "(0 = every stage of a batch in order on its own stream)")
    ap.add_argument("--walk-prio", type=int, default=0,
                    help="1: the pipelined walk on a high-priority stream over all CUs instead of --walk-cus CUs")
    ap.add_argument("--unmask-streams", type=int, default=1)
    ap.add_argument("--staged", type=int, default=1,
                    help="split pipeline staged by the host: walk, wait for it, then the unmask, so "
                         "consecutive unmasks follow each other on the unmask stream with no dependency "
                         "packet, event or empty check kernel between them; 0 = wsc_decode_split")
    ap.add_argument("--unmask-rest", action="store_true", help="mask the unmask streams to the CUs the walk does not use")
    ap.add_argument("--no-echo", action="store_true", help="skip the configs[0] loopback echo lines")
    ap.add_argument("--no-config3", action="store_true",
                    help="skip the BASELINE configs[3] line (1 M x 4 KiB frames per GPU dealt round-robin)")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the device-time lines for BASELINE.json configs[1], [2], [4]")
    ap.add_argument("--prewarm-ms", type=float, default=200.0,
                    help="untimed decodes for this long before the warm-up steps, so the timed steps run at the "
                         "GPU's sustained clock (a 20-step run is ~7 ms: shorter than the clock ramp)")
    ap.add_argument("--dry-run", action="store_true",
                    help="control path only (rank launch, process group, barriers, max-over-ranks timing, the "
                         "JSON line) with a CPU stand-in step and no device work: the CPU test of --gpus N")
    return ap.parse_args()


def launch_ranks(n):
    """`--gpus N` without a launcher: start N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process -- before this process has touched a GPU -- and
    return its exit code.  Rank r binds device r (LOCAL_RANK)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def cpu_model():
    """the host CPU's model name (lscpu's "Model name", read from /proc/cpuinfo)"""
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, seconds, threads):
    """The reference's hot loop (websocket_frame.go:33-42) ported to C (oracle/go_unmask_port.c),
    over the WHOLE batch (every frame, 1 GiB of payload at the headline: far larger than the
    host's last-level cache, so it streams from DRAM like the reference would), in passes until
    `seconds` of wall time have elapsed.  threads > 1: frames split over that many threads (one
    poller goroutine per core)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as O
    lib = O.goport()
    ns = cfg["n_frames"]
    wire = cfg["wire"]
    off = np.ascontiguousarray(cfg["payload_off"][:ns], dtype=np.uint64)
    ln = np.ascontiguousarray(cfg["plen"][:ns], dtype=np.uint32)
    mk = np.ascontiguousarray(cfg["mask"][:ns], dtype=np.uint32)
    args = (wire.ctypes.data, off.ctypes.data, ln.ctypes.data, mk.ctypes.data, ns)
    passes, t0 = 0, time.perf_counter()
    while True:
        if threads == 1:
            lib.goport_unmask_frames(*args)
        else:
            lib.goport_unmask_frames_mt(*args, threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gib = passes * int(ln.sum()) / 2**30
    return gib / el, passes, el


def main():
    a = parse()
    # --gpus N is authoritative: without a launcher, start N ranks (nothing has touched a GPU
    # yet); under a launcher, its world size must be N
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU, rank r on device LOCAL_RANK; WSC_BENCH_BACKEND=gloo + a shared device is
    # only for rehearsing the N>1 control path on a 1-GPU box (the driver's N>1 runs use RCCL)
    backend = "gloo" if a.dry_run else os.environ.get("WSC_BENCH_BACKEND", "nccl")
    if a.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        return dry_run(a, dist, world, rank)
    n_dev = torch.cuda.device_count()
    if backend == "nccl" and local >= n_dev:
        print(f"bench.py: rank {rank} wants device {local} but {n_dev} are visible", file=sys.stderr)
        sys.exit(2)
    local = local % max(1, n_dev)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    cdev = dev if backend == "nccl" else torch.device("cpu")   # where the timing collectives live

    from netman_amd import codec as K
    from netman_amd import synth

    seed = synth.SEED_BASE + 1 + 1000 * rank
    cfg = synth.uniform_batch(a.frames, a.frame_bytes, a.frames_per_seg, seed=seed)
    n_bytes = len(cfg["wire"])
    n_segs = len(cfg["seg_off"]) - 1
    over = dict(max_batch_bytes=n_bytes + 4096, max_segs=n_segs, max_frames=a.frames + 16)
    if a.waves_per_cu:
        over["unmask_waves_per_cu"] = a.waves_per_cu
    P = max(1, a.pipeline)
    codecs, batches, keep = [], [], []
    for j in range(P):
        c = K.Codec(local, **over)
        t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev),
                 seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
                 st_out=torch.zeros(n_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                 seg_out=torch.zeros(n_segs * 32, dtype=torch.uint8, device=dev),
                 frames=torch.zeros((a.frames + 16) * 32, dtype=torch.uint8, device=dev),
                 summ=torch.zeros(32, dtype=torch.uint8, device=dev))
        codecs.append(c)
        keep.append(t)
        batches.append(c.make_batch(t["wire"], t["seg_off"], None, t["st_out"], t["seg_out"], t["frames"], t["summ"]))
    codec, batch = codecs[0], batches[0]
    streams = [torch.cuda.Stream(device=dev) for _ in range(P)]
    torch.cuda.synchronize()

    # correctness gate on the real workload before timing (size-independent property: the first
    # decode of every in-flight buffer must equal the numpy restatement on a sample of frames)
    ok = True
    for c, b, t in zip(codecs, batches, keep):
        c.decode(b)
        c.sync()
        host = t["wire"][: min(n_bytes, 64 * (a.frame_bytes + 14))].cpu().numpy().copy()
        k = int(np.searchsorted(cfg["payload_off"] + cfg["plen"], len(host), side="right"))
        ref = synth.unmask_reference(cfg["wire"][: len(host)], cfg["payload_off"][:k], cfg["plen"][:k], cfg["mask"][:k])
        end = int(cfg["payload_off"][k - 1] + cfg["plen"][k - 1])
        ok = ok and bool(np.array_equal(host[:end], ref[:end]))
        summ_h = t["summ"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
        ok = ok and int(summ_h["n_frames"]) == a.frames and int(summ_h["n_spans"]) == a.frames

    # split pipeline: one walk stream on the first walk_cus CUs, one unmask stream per in-flight
    # batch on the rest, so batch k+1's walk runs beside batch k's unmask and the unmasks' ramp
    # and tail overlap (tools/split_probe.py, profiles/r01_split_probe.log)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    split = P > 1 and (a.walk_prio or 0 < a.walk_cus < n_cu)
    n_dec = [1] * P   # decodes issued per in-flight buffer (the gate above did one each)
    if split:
        walk_st = codec.stream_create(priority=1) if a.walk_prio else codec.stream_create(K.cu_mask(range(a.walk_cus), n_cu))
        um = K.cu_mask(range(a.walk_cus, n_cu), n_cu) if a.unmask_rest else None
        unmask_st = [codec.stream_create(um) for _ in range(max(1, a.unmask_streams))]

    def run(steps, depth):
        # batch i goes to context i % depth: independent batches (chaining the unmasks with
        # events measured slower: 0.361 vs 0.352 ms per step)
        if split and depth == P and a.staged:
            # staged: batch i+1's walk is enqueued, the host waits for it (it runs beside batch
            # i's unmask), then batch i+1's unmask follows batch i's on the unmask stream with no
            # dependency packet between them
            for i in range(steps):
                j = i % depth
                codecs[j].decode_walk(batches[j], walk_st)
                codecs[j].walk_wait()
                codecs[j].decode_finish(batches[j], unmask_st[j % len(unmask_st)])
                n_dec[j] += 1
            return
        for i in range(steps):
            j = i % depth
            if split and depth == P:
                codecs[j].decode_split(batches[j], walk_st, unmask_st[j % len(unmask_st)])
            else:
                codecs[j].decode(batches[j], streams[j].cuda_stream)
            n_dec[j] += 1

    def timed(depth):
        run(a.warmup, depth)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(a.steps, depth)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # clock pre-warm (untimed, not counted as warm-up steps): ~prewarm_ms of the same decodes
    if a.prewarm_ms > 0:
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < a.prewarm_ms * 1e-3:
            run(16, P)
            torch.cuda.synchronize()
    el_single = timed(1) if P > 1 else None   # one batch in flight: the per-batch latency
    el = timed(P)
    # after the timed runs: each buffer was XORed n_dec times in place, so it must be the masked
    # wire (even) or the unmasked reference (odd) on the sampled frames
    for j, t in enumerate(keep):
        host = t["wire"][: min(n_bytes, 64 * (a.frame_bytes + 14))].cpu().numpy().copy()
        k = int(np.searchsorted(cfg["payload_off"] + cfg["plen"], len(host), side="right"))
        end = int(cfg["payload_off"][k - 1] + cfg["plen"][k - 1])
        want = synth.unmask_reference(cfg["wire"][: len(host)], cfg["payload_off"][:k], cfg["plen"][:k],
                                      cfg["mask"][:k]) if n_dec[j] % 2 else cfg["wire"][: len(host)]
        ok = ok and bool(np.array_equal(host[:end], want[:end]))
    # every decode of the run (gate, warm-up, timed) on every context: no capacity overflow and no
    # look-back timeout (sticky device bits, wsc_error_flags), and each buffer's last summary is OK
    err_bits = 0
    for c, t in zip(codecs, keep):
        err_bits |= c.error_flags()
        ok = ok and K.Codec.summary_status(t["summ"].cpu().numpy().copy()) == K.WSC_OK
    ok = ok and err_bits == 0
    if split:
        torch.cuda.synchronize()
        for s_ in [walk_st] + unmask_st:
            codec.stream_destroy(s_)
    if world > 1:
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    # per-kernel device time (hipEvents on the codec's launch stream)
    prof = codec.profile(batch, max(5, min(a.steps, 20)))

    payload = cfg["payload_bytes"]
    value = payload * world * a.steps / el / 2**30   # all ranks' payload / max-over-ranks wall time
    hdr = 14 if a.frame_bytes > 65535 else (8 if a.frame_bytes > 125 else 6)
    alg_bytes = a.frames * (2 * a.frame_bytes + hdr + RECORD_BYTES)
    unmask_ms = prof["unmask"]
    achieved = alg_bytes / (unmask_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            pm = json.load(open(PMC_FILE))
            if pm.get("frames") == a.frames and pm.get("frame_bytes") == a.frame_bytes:
                traffic = pm.get("unmask_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "GiB/s masked WebSocket payload unmasked, device-resident, 64 KiB-frame batch",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded masked BIN frames, uniform random payload and masks)",
        "config": {"workload": f"{a.frames} x {a.frame_bytes} B masked BIN frames per GPU "
                               f"({payload / 2**30:.3f} GiB payload, {hdr} B headers, "
                               f"{a.frames_per_seg} frames per connection segment), in-place unmask",
                   "frames_per_gpu": a.frames, "frame_bytes": a.frame_bytes,
                   "segments_per_gpu": n_segs, "parallelism": f"shard{world}",
                   "batches_in_flight": P,
                   "pipeline": (f"split: walk on {'a high-priority stream over all CUs' if a.walk_prio else 'a stream masked to ' + str(a.walk_cus) + ' CUs'}, unmask (+ UTF-8 check when text was deferred) on "
                                f"{len(unmask_st)} stream(s) over "
                                f"{'the other ' + str(n_cu - a.walk_cus) if a.unmask_rest else 'all ' + str(n_cu)} CUs") if split
                               else "each batch in order on its own stream"},
        "parity_ok": ok,
        "device_error_flags": err_bits,
        "single_batch": None if el_single is None else {
            "ms_per_step": round(el_single / a.steps * 1e3, 4),
            "gib_s": round(cfg["payload_bytes"] * world * a.steps / el_single / 2**30, 2)},
        "kernel_ms": {k: round(v, 5) for k, v in prof.items()},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "k_unmask", "alg_bytes_per_launch": alg_bytes},
    }
    solo = world == 1   # the extra lines (host-inclusive, other configs, encode, echo, CPU baseline) are N=1 only
    if not a.no_config3:
        out["configs3_dealt"] = config3_dealt(a, torch, dist, K, synth, world, rank, dev, cdev)
    if solo and not a.no_host_inclusive:
        out["host_inclusive"] = host_inclusive(codec, cfg, K)
        # one copy stream per direction and three piece-sized contexts: 42.3 GiB/s on both runs of
        # profiles/r05/ab4_hi_*.log (2 contexts: 33.9-43.4; more copy streams per direction: slower)
        out["host_inclusive_pipelined"] = host_inclusive_pipelined(torch, codecs, streams, cfg, K, dir_streams=True, nbuf=3)
        out["host_inclusive_zero_copy"] = host_inclusive_zero_copy(torch, codecs, streams, cfg, K)
    for c in codecs:
        c.close()
    if solo and not a.no_other_configs:
        del keep, batches
        torch.cuda.empty_cache()
        out["other_configs"] = other_configs(torch, K, synth)
        out["encode"] = encode_configs(torch, K, synth)
    if solo and not a.no_echo:
        out["echo"] = echo_configs(with_cpu=not a.no_cpu)
    if solo and not a.no_cpu and a.cpu_seconds > 0:
        # every core this process may run on (the box's CPU share); 1 core = one poller goroutine
        threads = min(256, len(os.sched_getaffinity(0)))
        v1, p1, e1 = cpu_baseline(cfg, a.cpu_seconds / 3, 1)
        vm, pm_, em = cpu_baseline(cfg, a.cpu_seconds * 2 / 3, threads)
        out["cpu_baseline"] = {"value": round(vm, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                               "sample": f"the whole headline batch ({a.frames} frames, "
                                         f"{cfg['payload_bytes'] / 2**30:.2f} GiB payload, DRAM-resident), "
                                         f"{pm_} passes in {em:.1f} s on {threads} threads; "
                                         f"C port of websocket_frame.go:33-42 (Go absent)",
                               "value_1core": round(v1, 3), "cpu_model": cpu_model(),
                               "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def dry_run(a, dist, world, rank):
    """The control path of a --gpus N run with a CPU stand-in step (XOR of a 1 MiB buffer): the
    barriers, the max-over-ranks wall time and the JSON line, n_gpus = world.  No device work."""
    import torch
    buf = np.frombuffer(np.random.default_rng(rank).bytes(1 << 20), np.uint8).copy()

    def step():
        np.bitwise_xor(buf, np.uint8(0x5A), out=buf)

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        ranks = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(ranks, op=dist.ReduceOp.SUM)
        rank_sum = int(ranks.item())
    else:
        rank_sum = 0
    if rank == 0:
        print(json.dumps({"metric": "dry run (control path only, no device work)", "value": None,
                          "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(el / max(1, a.steps) * 1e3, 4), "rank_sum": rank_sum,
                          "data": "dry run"}))
    if world > 1:
        dist.destroy_process_group()


def config3_dealt(a, torch, dist, K, synth, world, rank, dev, cdev):
    """BASELINE.json configs[3] at N GPUs: ONE global batch of N x 1 M masked 4 KiB BIN frames
    (16 frames per connection segment; 8 M frames = 32 GiB at N = 8) whose segments are dealt
    round-robin to the ranks (shard.assign_segments: segment g -> rank g mod N), so every rank
    decodes its own 1 M-frame, 4 GiB shard -- independent, no collective on the data path.  Each
    rank decodes its shard back to back on one stream, two contexts in turn (below: the split
    pipeline measured slower here); the step time is the max over ranks; value = all ranks'
    payload x steps / that time.  Per-rank times are reported.  torch.distributed is used for
    the barriers, the max and the gather only."""
    per_rank, size, fps = 1 << 20, 4096, 16
    cfg = synth.dealt_uniform_batch(per_rank * world, size, fps, seed=synth.SEED_BASE + 3, world=world, rank=rank)
    n_bytes, n_segs, nf = len(cfg["wire"]), len(cfg["seg_off"]) - 1, cfg["n_frames"]
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    cs, bs, ts = [], [], []
    for j in range(2):
        c = K.Codec(dev.index, max_batch_bytes=n_bytes + 4096, max_segs=n_segs, max_frames=nf + 16)
        t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev),
                 seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
                 st=torch.zeros(n_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                 so=torch.zeros(n_segs * 32, dtype=torch.uint8, device=dev),
                 fr=torch.zeros((nf + 16) * 32, dtype=torch.uint8, device=dev),
                 sm=torch.zeros(32, dtype=torch.uint8, device=dev))
        cs.append(c)
        ts.append(t)
        bs.append(c.make_batch(t["wire"], t["seg_off"], None, t["st"], t["so"], t["fr"], t["sm"]))
    # serial decodes on one stream (each context's walk + unmask in turn) by default: with 1 M
    # frames the walk is 54 us on the whole chip, and beside the unmask (split pipeline) it took
    # CUs and bandwidth from it -- tools/c3_ab.sh: serial 2,799 GiB/s, split with the walk on
    # 128 / 48 / 16 CUs 2,685-2,710 / 2,438-2,444 / 2,112-2,129 (WSC_C3_SERIAL=0 and
    # WSC_C3_WALK_CUS select the split form)
    walk_cus = int(os.environ.get("WSC_C3_WALK_CUS", "0")) or min(n_cu // 2, max(16, (n_segs + 255) // 256))
    serial = os.environ.get("WSC_C3_SERIAL", "1") == "1"
    ws = cs[0].stream_create(K.cu_mask(range(walk_cus), n_cu))
    us = cs[0].stream_create(None)
    n_dec = [0, 0]

    def run(k):
        for i in range(k):
            if serial:
                cs[i % 2].decode(bs[i % 2], us)
            else:
                cs[i % 2].decode_split(bs[i % 2], ws, us)
            n_dec[i % 2] += 1

    run(a.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # parity on a sample (the first 64 frames of each buffer: unmasked after an odd number of
    # decodes, the masked wire after an even one) + every decode's device error bits
    m = int(cfg["payload_off"][63] + cfg["plen"][63])
    ref = synth.unmask_reference(cfg["wire"][:m], cfg["payload_off"][:64], cfg["plen"][:64], cfg["mask"][:64])
    ok = True
    for j in range(2):
        got = ts[j]["wire"][:m].cpu().numpy()
        ok = ok and bool(np.array_equal(got, ref if n_dec[j] % 2 else cfg["wire"][:m]))
        ok = ok and cs[j].error_flags() == 0
        summ = ts[j]["sm"].cpu().numpy().copy().view(K.SUMMARY_DTYPE)[0]
        ok = ok and int(summ["n_frames"]) == nf
    cs[0].stream_destroy(ws)
    cs[0].stream_destroy(us)
    for c in cs:
        c.close()
    del ts, bs
    torch.cuda.empty_cache()
    times = [el]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        times = [float(x.item()) for x in g]
        okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    tmax = max(times)
    return {"workload": f"{per_rank * world} x {size} B masked BIN frames ({fps} per connection segment), "
                        f"segments dealt round-robin to {world} GPU(s): {per_rank} frames = "
                        f"{cfg['payload_bytes'] / 2**30:.1f} GiB per GPU",
            "gib_s": round(cfg["payload_bytes"] * world * a.steps / tmax / 2**30, 1),
            "ms_per_step": round(tmax / a.steps * 1e3, 4),
            "per_rank_ms_per_step": [round(x / a.steps * 1e3, 4) for x in times],
            "n_gpus": world, "scaling": "weak", "parity_ok": ok,
            "mode": "serial decodes on one stream" if serial else f"split pipeline, walk on {walk_cus} CUs"}


def other_configs(torch, K, synth, only=None):
    """The other single-GPU BASELINE.json configs, beside the headline; parity for each is in
    tests/test_gpu_parity.py.  `ms`: one batch in flight -- back-to-back decodes of one batch on
    one stream (each walk waits for the previous unmask), hipEvents around 100 decodes after 30
    warm-up decodes (a 20-decode burst measured ~10 % slow at configs[1]: the GPU clock ramp);
    `walk_ms` / `unmask_ms`: per-kernel device time (wsc_profile hipEvents, median of 10);
    `pipelined_*`: two batches in flight through the staged split pipeline the headline runs
    (walk on a CU-masked stream, the host waits for it, then the unmask), wall time of 60 steps
    after 20 warm-up steps, best of the PIPELINE_SPLITS CU partitions and the serial order (reported).  `frac`: the
    decode's algorithmic bytes (2 x payload + header + 32 B record per frame) per second over
    the 8 TB/s HBM peak."""
    dev = torch.device("cuda", torch.cuda.current_device())
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    res = {}
    cases = [("configs[1] 1M x 1 KiB BIN, 16 frames/segment", lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1), False),
             ("configs[1] 1M x 1 KiB BIN, 1 frame/segment", lambda: synth.uniform_batch(1 << 20, 1024, 1, seed=synth.SEED_BASE + 1), False),
             ("configs[2] 256k mixed 125 B / 64 KiB / 1 MiB (p~1/size)", lambda: synth.mixed_batch(), False),
             ("configs[2] 256k mixed, 1 frame/segment", lambda: synth.mixed_batch(frames_per_seg=1), False),
             ("configs[3] one GPU's shard: 1M x 4 KiB BIN, 16 frames/segment",
              lambda: synth.uniform_batch(1 << 20, 4096, 16, seed=synth.SEED_BASE + 3), False),
             ("configs[4] 64k connections x fragmented message, reassembled (COMPACT)", lambda: synth.fragmented_batch(), True),
             ("TEXT 16384 x 64 KiB valid UTF-8 (1-4 byte characters), 4 frames/segment",
              lambda: synth.text_batch(16384, 65536, 4, seed=synth.SEED_BASE + 7), False),
             ("TEXT 262144 x 1 KiB valid UTF-8, 16 frames/segment",
              lambda: synth.text_batch(262144, 1024, 16, seed=synth.SEED_BASE + 8), False)]
    for name, make, compact in cases:
        if only and not any(o in name for o in only):
            continue
        cfg = make()
        n = len(cfg["seg_off"]) - 1

        def one():
            c = K.Codec(dev.index, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=n, max_frames=cfg["n_frames"] + 16)
            t = dict(wire=torch.from_numpy(cfg["wire"]).to(dev),
                     seg_off=torch.from_numpy(cfg["seg_off"].view(np.int64)).to(dev),
                     st=torch.zeros(n * K.STATE_BYTES, dtype=torch.uint8, device=dev), so=torch.zeros(n * 32, dtype=torch.uint8, device=dev),
                     fr=torch.zeros((cfg["n_frames"] + 16) * 32, dtype=torch.uint8, device=dev),
                     sm=torch.zeros(32, dtype=torch.uint8, device=dev))
            if compact:
                t["arena"] = torch.zeros(len(cfg["wire"]) + 64, dtype=torch.uint8, device=dev)
                t["fd"] = torch.zeros(cfg["n_frames"] + 16, dtype=torch.int64, device=dev)
            b = c.make_batch(t["wire"], t["seg_off"], None, t["st"], t["so"], t["fr"], t["sm"], compact=compact,
                             arena=t.get("arena"), frame_dst=t.get("fd"))
            return c, t, b

        c, t, b = one()
        st = torch.cuda.Stream(device=dev)
        # An in-place decode leaves the payload unmasked, so a TEXT batch decoded again would be
        # validated as garbage (1007 at its first frame, the re-mask path): every TEXT decode starts
        # from the pristine masked wire (device copy, outside the timed events)
        text = name.startswith("TEXT")
        pristine = t["wire"].clone() if text else None

        def restore():
            if text:
                with torch.cuda.stream(st):
                    t["wire"].copy_(pristine)

        for _ in range(30):
            restore()
            c.decode(b, st.cuda_stream)
        torch.cuda.synchronize()
        if text:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
            for e0, e1 in ev:
                restore()
                e0.record(st)
                c.decode(b, st.cuda_stream)
                e1.record(st)
            torch.cuda.synchronize()
            tot = float(sum(e0.elapsed_time(e1) for e0, e1 in ev)) / 20
            seg = t["so"].view(-1, 32)[:, 20:24].contiguous().view(torch.int32).cpu()   # close_code
            ok = int((seg != 0).sum()) == 0   # valid text everywhere: no segment closed (1007)
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(100):
                c.decode(b, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            tot = float(e0.elapsed_time(e1)) / 100
            ok = True
        ok = ok and c.error_flags() == 0
        p = []
        for _ in range(10):
            restore()
            torch.cuda.synchronize()
            p.append(c.profile(b, 1))
        um = float(np.median([q["unmask"] for q in p]))
        wk = float(np.median([q["walk"] for q in p]))
        u8 = float(np.median([q["u8"] for q in p]))
        hdr = np.where(cfg["plen"] <= 125, 6, np.where(cfg["plen"] <= 65535, 8, 14))
        alg = int((2 * cfg["plen"].astype(np.int64) + hdr + 32).sum())
        if text:   # the pipelined leg re-decodes its batches in place: not measurable for TEXT
            res[name] = {"gib_s": round(cfg["payload_bytes"] / (tot * 1e-3) / 2**30, 1), "ms": round(tot, 4),
                         "frac": round(alg / (tot * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
                         "walk_ms": round(wk, 4), "unmask_ms": round(um, 4), "u8_ms": round(u8, 4),
                         "unmask_gb_s": round(alg / (um * 1e-3) / 1e9, 1),
                         "timing": "hipEvents around each decode of the pristine batch (restored in between)",
                         "frames": int(cfg["n_frames"]), "payload_bytes": int(cfg["payload_bytes"]), "alg_bytes": alg,
                         "device_errors": not ok}
            c.close()
            del t
            torch.cuda.empty_cache()
            continue
        # two batches in flight through the staged split pipeline.  The split of the CUs between
        # the walk and the unmask is tuned per config (tools/staged_probe.py): a latency-bound walk
        # that shares its SIMDs with the unmask's waves slows ~8x, so for many-frame configs the
        # unmask is best kept off the walk's CUs; for few-frame ones the unmask wants every CU
        torch.cuda.synchronize()
        c2, t2, b2 = one()
        pair = [(c, b), (c2, b2)]
        # the one-batch leg re-decodes ONE buffer, whose tail the caches may still hold from the
        # previous pass; the same back-to-back decodes alternating over two buffers (one context,
        # one stream) show what that reuse is worth
        for _ in range(10):
            c.decode(b2, st.cuda_stream)
        e0.record(st)
        for i in range(100):
            c.decode(b if i % 2 == 0 else b2, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        two_ms = float(e0.elapsed_time(e1)) / 100
        best, serial_ms = None, float("nan")
        for wcus, rest in PIPELINE_SPLITS:
            if wcus < 0:
                ws = us = c.stream_create(None)
            else:
                ws = c.stream_create(priority=1) if wcus == 0 else c.stream_create(K.cu_mask(range(wcus), n_cu))
                us = c.stream_create(K.cu_mask(range(wcus, n_cu), n_cu) if rest else None)

            def staged(k):
                for i in range(k):
                    cx, bx = pair[i % 2]
                    if wcus < 0:   # serial order: stream order alone separates the two batches, so
                        c.decode(bx, us)   # one context's scratch serves both (no second copy in the caches)
                        continue
                    cx.decode_walk(bx, ws)
                    cx.walk_wait()
                    cx.decode_finish(bx, us)

            staged(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            staged(60)
            torch.cuda.synchronize()
            pms = (time.perf_counter() - t0) / 60 * 1e3
            c.stream_destroy(ws)
            if us != ws:
                c.stream_destroy(us)
            if wcus < 0:
                serial_ms = pms
            if best is None or pms < best[0]:
                best = (pms, wcus, rest)
        pms, wcus, rest = best
        ok = ok and c.error_flags() == 0 and c2.error_flags() == 0
        res[name] = {"gib_s": round(cfg["payload_bytes"] / (tot * 1e-3) / 2**30, 1), "ms": round(tot, 4),
                     "frac": round(alg / (tot * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
                     "walk_ms": round(wk, 4), "unmask_ms": round(um, 4), "unmask_gb_s": round(alg / (um * 1e-3) / 1e9, 1),
                     "pipelined_gib_s": round(cfg["payload_bytes"] / (pms * 1e-3) / 2**30, 1),
                     "pipelined_ms_per_batch": round(pms, 4),
                     "pipelined_frac": round(alg / (pms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
                     "pipelined_walk_cus": wcus if wcus > 0 else ("all, high-priority stream" if wcus == 0 else
                                                                  "serial: walks and unmasks in order on one stream"),
                     "pipelined_unmask_cus": "the other CUs" if rest else "all",
                     # the best candidate can be the serial order (no overlap at all): say so, and
                     # give the serial time on its own (round-5 ADVICE)
                     "pipelined_is_serial": wcus < 0,
                     "serial_ms_per_batch": round(serial_ms, 4),
                     "two_buffers_ms": round(two_ms, 4),
                     "frames": int(cfg["n_frames"]), "payload_bytes": int(cfg["payload_bytes"]), "alg_bytes": alg,
                     "device_errors": not ok}
        c.close()
        c2.close()
        del t, t2
        torch.cuda.empty_cache()
    return res


def encode_configs(torch, K, synth):
    """Batched server->client framing (wsc_encode, websocket_ctrl.go:23-70) of the decoded
    payloads of a batch -- the echo path's outbound half: device time (torch events on the launch
    stream around bursts of 20 back-to-back encodes, median of 5) of k_encode_scan +
    k_encode_copy, algorithmic bytes = payload read +
    frames written + 24 B descriptor + 8 B offset per message."""
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}
    cases = [("16384 x 64 KiB BIN (echo of the headline batch)", lambda: synth.uniform_batch(16384, 65536, 4, seed=synth.SEED_BASE + 1)),
             ("1M x 1 KiB BIN (echo of configs[1])", lambda: synth.uniform_batch(1 << 20, 1024, 16, seed=synth.SEED_BASE + 1))]
    for name, make in cases:
        cfg = make()
        n = int(cfg["n_frames"])
        msgs = np.zeros(n, K.OUT_MSG_DTYPE)
        msgs["src_off"] = cfg["payload_off"]
        msgs["len"] = cfg["plen"]
        msgs["first_byte"] = 0x82
        hl = np.where(cfg["plen"] <= 125, 2, np.where(cfg["plen"] <= 65535, 4, 10)).astype(np.int64)
        total = int((cfg["plen"].astype(np.int64) + hl).sum())
        c = K.Codec(dev.index, max_batch_bytes=len(cfg["wire"]) + 4096, max_segs=1024, max_frames=n + 16)
        src = torch.from_numpy(cfg["wire"]).to(dev)
        d_msgs = torch.from_numpy(msgs.view(np.uint8).copy()).to(dev)
        d_out = torch.empty(total + 4096, dtype=torch.uint8, device=dev)
        d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        st = torch.cuda.Stream(device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        times = []
        # back-to-back encodes, as other_configs times decodes: 20 warm-up, then hipEvents around
        # bursts of 20 (a launch-sync-launch loop left the chip idle between encodes and timed
        # each one from a cold clock: ~30 us more than the kernel sum at 1 KiB)
        with torch.cuda.stream(st):
            for _ in range(20):
                c.encode(d_msgs, n, src, len(cfg["wire"]), d_out, total + 4096, d_off, st.cuda_stream)
        for it in range(5):
            with torch.cuda.stream(st):
                ev[0].record(st)
                for _ in range(20):
                    c.encode(d_msgs, n, src, len(cfg["wire"]), d_out, total + 4096, d_off, st.cuda_stream)
                ev[1].record(st)
            ev[1].synchronize()
            times.append(ev[0].elapsed_time(ev[1]) / 20)
        ok = int(d_off[-1].item()) == total
        # spot check: the first frame's header + payload and the last frame's payload end
        o = d_out[: 16].cpu().numpy()
        L = int(cfg["plen"][0])
        exp_hdr = bytes([0x82, 127]) + L.to_bytes(8, "big") if L > 65535 else (bytes([0x82, 126]) + L.to_bytes(2, "big") if L > 125 else bytes([0x82, L]))
        ok = ok and o[: len(exp_hdr)].tobytes() == exp_hdr
        p0 = int(cfg["payload_off"][0])
        ok = ok and bool(np.array_equal(d_out[len(exp_hdr): len(exp_hdr) + 64].cpu().numpy(), cfg["wire"][p0:p0 + 64]))
        ms = float(np.median(times))
        alg = int(cfg["payload_bytes"]) + total + 32 * n
        res[name] = {"ms": round(ms, 4), "gb_s": round(alg / (ms * 1e-3) / 1e9, 1),
                     "payload_gib_s": round(cfg["payload_bytes"] / (ms * 1e-3) / 2**30, 1),
                     "frames": n, "out_bytes": total, "alg_bytes": alg, "check_ok": ok}
        c.close()
        del src, d_msgs, d_out, d_off
        torch.cuda.empty_cache()
    return res


def echo_configs(with_cpu=True):
    """configs[0]: examples/websocket echo on loopback, rebuilt around a pluggable decoder
    (tools/echo_harness.hpp; the Go reference server cannot run here).  gpu = tools/ws_echo
    (libwscodec wsc_session: recv straight into pinned staging, round r+1 submitted to the device
    while round r is echoed); gpu_sync = the same with one synchronous decode per round; gpu_blocking_wait =
    gpu with the session's completion sleeping on a blocking-sync event (WSC_SESSION_BLOCKING_WAIT)
    instead of spinning; cpu = oracle/_build/ws_echo_cpu,
    the reference's frame-at-a-time decode ported to C++ (cpu_baseline leg, kind "port").  Each
    run is a separate process; msgs/s and GiB/s of echoed payload, every byte checked.  P pollers
    (netman runs NumCPU, eventloop/event.go:33-37): connection i on poller i % P, each poller its
    own decoder -- for the GPU its own wsc_session on the one device.  One read(2) takes at most
    4 MiB per connection and round unless a row says otherwise (--read-bytes).  Every run also
    reports the server's CPU seconds (the whole process minus the client threads: pollers plus the
    HIP runtime's and any batching thread) and those per GiB echoed -- both servers are client-bound
    on loopback from 4 pollers on, so GiB/s cannot tell them apart; the CPU the server spends can."""
    import subprocess
    gpu = os.path.join(ROOT, "tools", "ws_echo")
    cpu = os.path.join(ROOT, "oracle", "_build", "ws_echo_cpu")
    runs = [("1 conn x 4000 x 64 KiB (configs[0])", ["--conns", "1", "--frames", "4000", "--size", "65536"],
             ["gpu", "gpu_sync", "cpu_port"])]
    for P in (1, 4, 8):
        runs.append((f"64 conns x 200 x 64 KiB, {P} poller(s)", ["--conns", "64", "--frames", "200", "--size", "65536",
                                                                  "--client-threads", "4", "--pollers", str(P)],
                     ["gpu", "gpu_blocking_wait", "cpu_port"]))
        # the same traffic with at most 512 KiB per read(2) (--read-bytes): more, smaller rounds.  The
        # echo is client-bound from 4 pollers on (ECHO_TIMING: the pollers' loops are busy ~1/3 of
        # the run), and how early the replies go out moves both servers by 10-40 %
        runs.append((f"64 conns x 200 x 64 KiB, {P} poller(s), 512 KiB reads", ["--conns", "64", "--frames", "200", "--size", "65536",
                                                                                "--client-threads", "4", "--pollers", str(P),
                                                                                "--read-bytes", "524288"],
                     ["gpu", "cpu_port"]))
        runs.append((f"64 conns x 2000 x 1 KiB, {P} poller(s)", ["--conns", "64", "--frames", "2000", "--size", "1024",
                                                                 "--client-threads", "4", "--pollers", str(P)],
                     ["gpu", "gpu_sync", "cpu_port"]))
    # clients half-close after their last frame (the EOF rule: every message echoed before Close())
    runs.append(("64 conns x 200 x 64 KiB, 4 pollers, clients shutdown(SHUT_WR) after the last frame",
                 ["--conns", "64", "--frames", "200", "--size", "65536", "--client-threads", "4", "--pollers", "4",
                  "--shutdown"], ["gpu", "cpu_port"]))
    bins = {"gpu": (gpu, []), "gpu_sync": (gpu, ["--sync"]), "gpu_blocking_wait": (gpu, ["--blocking-wait"]),
            "cpu_port": (cpu, [])}

    def one(exe, args):
        try:
            p = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            d = json.loads(line[-1]) if line else {"ok": False, "error": p.stderr[-300:]}
            return {k: d.get(k) for k in ("ok", "gib_s", "msgs_per_s", "seconds", "rounds", "server_cpu_s",
                                          "server_cpu_s_per_gib", "poller_cpu_s_per_gib", "client_cpu_s", "error")}
        except Exception as e:   # the echo lines are reported beside the metric, never fatal
            return {"ok": False, "error": repr(e)[:200]}

    # loopback echo rates move by 10-25 % run to run on one box: every row runs REPS times with
    # its kinds interleaved (gpu, sync, cpu, gpu, ...) so drift hits them alike; the median run is
    # reported with all runs' rates beside it
    REPS = 3
    res = {}
    for name, args, kinds in runs:
        kinds = [k for k in kinds if (k != "cpu_port" or with_cpu)]
        got = {k: [] for k in kinds}
        for _ in range(REPS):
            for kind in kinds:
                exe, extra = bins[kind]
                got[kind].append(one(exe, args + extra) if os.path.exists(exe) else None)
        row = {}
        for kind, rs in got.items():
            good = sorted([r for r in rs if r and r.get("ok")], key=lambda r: r["gib_s"])
            if not good:
                row[kind] = next((r for r in rs if r), None)
                continue
            row[kind] = dict(good[len(good) // 2], gib_s_runs=[r["gib_s"] for r in rs if r and r.get("ok")],
                             # what the server costs its host per GiB echoed, whatever the clients allow
                             # through loopback: the median over the runs, beside the median run's rate
                             server_cpu_s_per_gib_median=float(np.median([r["server_cpu_s_per_gib"] for r in good])))
            if len(good) < len(rs):
                row[kind]["failed_runs"] = len(rs) - len(good)
        res[name] = row
    return res


def host_inclusive(codec, cfg, K):
    """wsc_decode_host on pinned host buffers: H2D of the wire, decode, D2H of the unmasked wire
    and the records (reported in DESIGN.md, never as `value`)."""
    lib = K.load_library()
    n = len(cfg["wire"])
    p = C.c_void_p()
    if lib.wsc_host_alloc(n, C.byref(p)) != 0:
        return None
    try:
        buf = np.frombuffer((C.c_uint8 * n).from_address(p.value), dtype=np.uint8)
        buf[:] = cfg["wire"]
        t0 = time.perf_counter()
        iters = 3
        for _ in range(iters):
            codec.decode_host(buf, cfg["seg_off"])
        el = (time.perf_counter() - t0) / iters
        return {"gib_s": round(cfg["payload_bytes"] / el / 2**30, 2), "ms_per_batch": round(el * 1e3, 2),
                "note": "pinned host wire -> H2D -> decode -> D2H wire+records, synchronous"}
    finally:
        lib.wsc_host_free(p)


def host_inclusive_pipelined(torch, codecs, streams, cfg, K, chunks=16, iters=3, dir_streams=False, nbuf=0,
                             copy_streams=1, kcopy=0):
    """The same batch from pinned host memory, cut at segment boundaries into `chunks` pieces that
    alternate between the in-flight contexts/streams: H2D of piece i+1 overlaps the decode and
    the D2H of piece i (PCIe is full duplex).  Output: unmasked wire + frame records in pinned
    host memory.  Reported in DESIGN.md, never as `value`.  nbuf > len(codecs): that many piece-
    sized contexts of its own; copy_streams: streams per copy direction (dir_streams), piece i on
    stream i % copy_streams (the copy engines a stream lands on decide whether H2D and D2H overlap).
    kcopy (each piece's copies on its decode stream): 1 = the wire's H2D by a kernel reading the
    pinned host buffer (wsc_kcopy), 2 = also the D2H of the wire and the records by kernels."""
    own = []
    if nbuf > len(codecs):
        n_segs_all = len(cfg["seg_off"]) - 1
        piece_bytes = int(cfg["seg_off"][min(n_segs_all, (n_segs_all + chunks - 1) // chunks + 1)]) * 2 + 4096
        own = [K.Codec(0, max_batch_bytes=piece_bytes, max_segs=n_segs_all // chunks + 16,
                       max_frames=int(codecs[0].cfg.max_frames)) for _ in range(nbuf)]
        codecs = own
        streams = [torch.cuda.Stream() for _ in range(nbuf)]
    try:
        return _host_inclusive_pipelined(torch, codecs, streams, cfg, K, chunks, iters, dir_streams, copy_streams, kcopy)
    finally:
        for c in own:
            c.close()


def _host_inclusive_pipelined(torch, codecs, streams, cfg, K, chunks, iters, dir_streams, copy_streams, kcopy=0):
    P = len(codecs)
    if P < 2:
        return None
    dev = torch.device("cuda", torch.cuda.current_device())
    hold = []   # wsc_host_alloc blocks (kcopy: buffers a kernel reads / writes by their host address)

    def host_buf(nbytes):
        if not kcopy:
            return torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        lib = K.load_library()
        p = C.c_void_p()
        if lib.wsc_host_alloc(nbytes, C.byref(p)) != 0:
            raise RuntimeError("wsc_host_alloc")
        hold.append(p)
        return torch.from_numpy(np.frombuffer((C.c_uint8 * nbytes).from_address(p.value), dtype=np.uint8))

    wire_h = host_buf(len(cfg["wire"]))
    wire_h.copy_(torch.from_numpy(cfg["wire"]))
    out_h = host_buf(len(cfg["wire"]))
    so = cfg["seg_off"].astype(np.int64)
    n_segs = len(so) - 1
    cuts = [int(round(i * n_segs / chunks)) for i in range(chunks + 1)]
    pieces = []
    for i in range(chunks):
        s0, s1 = cuts[i], cuts[i + 1]
        if s1 <= s0:
            continue
        rel = torch.from_numpy((so[s0:s1 + 1] - so[s0]).copy()).pin_memory()
        pieces.append((int(so[s0]), int(so[s1]), s1 - s0, rel))
    max_bytes = max(b - a for a, b, _, _ in pieces)
    max_segs = max(k for _, _, k, _ in pieces)
    max_frames = int(codecs[0].cfg.max_frames)
    bufs = []
    for j in range(P):
        bufs.append(dict(wire=torch.empty(max_bytes + 16, dtype=torch.uint8, device=dev),
                         seg_off=torch.empty(max_segs + 1, dtype=torch.int64, device=dev),
                         st=torch.empty(max_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                         so=torch.empty(max_segs * 32, dtype=torch.uint8, device=dev),
                         fr=torch.empty(max_frames * 32, dtype=torch.uint8, device=dev),
                         sm=torch.empty(32, dtype=torch.uint8, device=dev)))
    rec_h = [host_buf(max_frames * 32) for _ in pieces]
    rec_n = [0] * len(pieces)
    for i, (a0, a1, k, _) in enumerate(pieces):
        rec_n[i] = int(np.count_nonzero((cfg["payload_off"] >= a0) & (cfg["payload_off"] < a1)))

    # one stream per PCIe direction (dir_streams): H2D of piece i+1 queued on its own stream can run
    # beside piece i's D2H on another, instead of queueing behind it on the piece's stream; events
    # order buffer reuse (H2D into buffer j waits for the D2H out of it) and each decode
    h2ds = [torch.cuda.Stream(device=dev) for _ in range(copy_streams)] if dir_streams else []
    d2hs = [torch.cuda.Stream(device=dev) for _ in range(copy_streams)] if dir_streams else []
    ev_free = [None] * P

    def one_pass():
        for i, (a0, a1, k, rel) in enumerate(pieces):
            j = i % P
            st, b = streams[j], bufs[j]
            batch = codecs[j].make_batch(b["wire"], b["seg_off"][: k + 1], None, b["st"], b["so"], b["fr"],
                                         b["sm"], n_bytes=a1 - a0)
            if dir_streams:
                h2d, d2h = h2ds[i % copy_streams], d2hs[i % copy_streams]
                with torch.cuda.stream(h2d):
                    if ev_free[j] is not None:
                        h2d.wait_event(ev_free[j])
                    b["wire"][: a1 - a0].copy_(wire_h[a0:a1], non_blocking=True)
                    b["seg_off"][: k + 1].copy_(rel, non_blocking=True)
                    ev_in = torch.cuda.Event()
                    ev_in.record(h2d)
                st.wait_event(ev_in)
                codecs[j].decode(batch, st.cuda_stream)
                ev_dec = torch.cuda.Event()
                ev_dec.record(st)
                with torch.cuda.stream(d2h):
                    d2h.wait_event(ev_dec)
                    out_h[a0:a1].copy_(b["wire"][: a1 - a0], non_blocking=True)
                    rec_h[i][: rec_n[i] * 32].copy_(b["fr"][: rec_n[i] * 32], non_blocking=True)
                    ev_free[j] = torch.cuda.Event()
                    ev_free[j].record(d2h)
                continue
            with torch.cuda.stream(st):
                if kcopy:
                    codecs[j].kcopy(b["wire"], wire_h.data_ptr() + a0, a1 - a0, st.cuda_stream)
                else:
                    b["wire"][: a1 - a0].copy_(wire_h[a0:a1], non_blocking=True)
                b["seg_off"][: k + 1].copy_(rel, non_blocking=True)
                codecs[j].decode(batch, st.cuda_stream)
                if kcopy >= 2:
                    codecs[j].kcopy(out_h.data_ptr() + a0, b["wire"], a1 - a0, st.cuda_stream)
                    codecs[j].kcopy(rec_h[i], b["fr"], rec_n[i] * 32, st.cuda_stream)
                else:
                    out_h[a0:a1].copy_(b["wire"][: a1 - a0], non_blocking=True)
                    rec_h[i][: rec_n[i] * 32].copy_(b["fr"][: rec_n[i] * 32], non_blocking=True)

    one_pass()
    torch.cuda.synchronize()
    ref = synth_unmask_prefix(cfg, 1 << 20)
    ok = bool(torch.equal(out_h[: len(ref)], torch.from_numpy(ref)))
    t0 = time.perf_counter()
    for _ in range(iters):
        one_pass()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / iters
    lib = K.load_library() if hold else None
    for p in hold:
        lib.wsc_host_free(p)
    return {"gib_s": round(cfg["payload_bytes"] / el / 2**30, 2), "ms_per_batch": round(el * 1e3, 2),
            "chunks": len(pieces), "streams": P, "copy_streams_per_direction": copy_streams if dir_streams else 0,
            "kcopy": kcopy, "parity_ok": ok,
            "note": "pinned host wire -> H2D -> decode -> D2H wire+records, pieces alternating over streams"
                    + (" (one stream per copy direction, events between them)" if dir_streams else " (each piece's copies on its decode stream)")}


def host_inclusive_zero_copy(torch, codecs, streams, cfg, K, chunks=16, iters=3):
    """Host-inclusive with the outbound copy done by the unmask itself: H2D of each piece's wire on
    the copy engine (stream j), walk on the device copy, then the COMPACT unmask writes each
    payload straight into a pinned, device-mapped host arena over PCIe -- the host receives the
    messages' bytes (headers stripped, wsc_session's COMPACT layout) and the records.  The next
    piece's H2D (copy engine, host -> device) runs while this piece's unmask writes device -> host:
    both PCIe directions busy at once, which the copy engines alone do not do for one process
    (profiles/r01_pcie_duplex.log).  Reported in DESIGN.md, never as `value`."""
    from netman_amd import synth
    P = len(codecs)
    if P < 2:
        return None
    lib = K.load_library()
    dev = torch.device("cuda", torch.cuda.current_device())
    wire_h = torch.from_numpy(cfg["wire"]).pin_memory()
    so = cfg["seg_off"].astype(np.int64)
    n_segs = len(so) - 1
    cuts = [int(round(i * n_segs / chunks)) for i in range(chunks + 1)]
    poff = cfg["payload_off"].astype(np.int64)
    plen = cfg["plen"].astype(np.int64)
    pieces, abase = [], 0
    for i in range(chunks):
        s0, s1 = cuts[i], cuts[i + 1]
        if s1 <= s0:
            continue
        a0, a1 = int(so[s0]), int(so[s1])
        sel = (poff >= a0) & (poff < a1)
        nb = int(plen[sel].sum())
        rel = torch.from_numpy((so[s0:s1 + 1] - so[s0]).copy()).pin_memory()
        pieces.append((a0, a1, s1 - s0, rel, abase, int(np.count_nonzero(sel))))
        abase += (nb + 15) // 16 * 16
    arena_bytes = abase + 64
    ap = C.c_void_p()
    if lib.wsc_host_alloc(arena_bytes, C.byref(ap)) != 0:
        return None
    try:
        arena_h = np.frombuffer((C.c_uint8 * arena_bytes).from_address(ap.value), dtype=np.uint8)
        max_bytes = max(p[1] - p[0] for p in pieces)
        max_segs = max(p[2] for p in pieces)
        max_frames = int(codecs[0].cfg.max_frames)
        bufs = []
        for j in range(P):
            bufs.append(dict(wire=torch.empty(max_bytes + 16, dtype=torch.uint8, device=dev),
                             seg_off=torch.empty(max_segs + 1, dtype=torch.int64, device=dev),
                             st=torch.empty(max_segs * K.STATE_BYTES, dtype=torch.uint8, device=dev),
                             so=torch.empty(max_segs * 32, dtype=torch.uint8, device=dev),
                             fr=torch.empty(max_frames * 32, dtype=torch.uint8, device=dev),
                             fd=torch.empty(max_frames, dtype=torch.int64, device=dev),
                             sm=torch.empty(32, dtype=torch.uint8, device=dev)))
        rec_h = [torch.empty(max(1, p[5]) * 32, dtype=torch.uint8).pin_memory() for p in pieces]

        def one_pass():
            for i, (a0, a1, k, rel, ab, nf) in enumerate(pieces):
                j = i % P
                st, b = streams[j], bufs[j]
                with torch.cuda.stream(st):
                    b["wire"][: a1 - a0].copy_(wire_h[a0:a1], non_blocking=True)
                    b["seg_off"][: k + 1].copy_(rel, non_blocking=True)
                    batch = codecs[j].make_batch(b["wire"], b["seg_off"][: k + 1], None, b["st"], b["so"], b["fr"],
                                                 b["sm"], compact=True, arena=None, frame_dst=b["fd"], n_bytes=a1 - a0)
                    batch.arena = ap.value + ab
                    codecs[j].decode(batch, st.cuda_stream)
                    rec_h[i][: nf * 32].copy_(b["fr"][: nf * 32], non_blocking=True)

        one_pass()
        torch.cuda.synchronize()
        # parity: the first piece's messages, in order, are the unmasked payloads
        a0, a1, _, _, ab, nf = pieces[0]
        k = min(nf, 64)
        ref = synth.unmask_reference(cfg["wire"][: int(poff[k - 1] + plen[k - 1])], cfg["payload_off"][:k],
                                     cfg["plen"][:k], cfg["mask"][:k])
        want = np.concatenate([ref[int(poff[i]):int(poff[i] + plen[i])] for i in range(k)])
        ok = bool(np.array_equal(arena_h[ab:ab + len(want)], want))
        ok = ok and all(c.error_flags() == 0 for c in codecs)
        t0 = time.perf_counter()
        for _ in range(iters):
            one_pass()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / iters
        return {"gib_s": round(cfg["payload_bytes"] / el / 2**30, 2), "ms_per_batch": round(el * 1e3, 2),
                "chunks": len(pieces), "streams": P, "parity_ok": ok,
                "note": "pinned host wire -> H2D (copy engine) -> walk -> COMPACT unmask writing the messages "
                        "into a pinned host arena over PCIe (+ records D2H), pieces alternating over streams"}
    finally:
        torch.cuda.synchronize()
        lib.wsc_host_free(ap)


def synth_unmask_prefix(cfg, n):
    from netman_amd import synth
    k = int(np.searchsorted(cfg["payload_off"] + cfg["plen"], n, side="right"))
    ref = synth.unmask_reference(cfg["wire"][:n], cfg["payload_off"][:k], cfg["plen"][:k], cfg["mask"][:k])
    end = int(cfg["payload_off"][k - 1] + cfg["plen"][k - 1])   # the k-th frame's payload end
    return np.ascontiguousarray(ref[:end])


if __name__ == "__main__":
    main()
