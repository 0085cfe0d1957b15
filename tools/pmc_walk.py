"""Per-launch HBM traffic of every decode kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of
tools/single_loop.py (one config per pair of runs), with the gfx950 correction MI355X_MICROARCH.md
prescribes for 16 B/lane reads (FETCH_SIZE x 2; WRITE_SIZE exact), next to each kernel's algorithmic
bytes.  bash tools/pmc_walk.sh gpurun_out/pmc c1 c11 c2 c4 && python tools/pmc_walk.py gpurun_out/pmc > profiles/pmc_walk_r03.json"""
import collections
import csv
import json
import os
import sys

# algorithmic bytes per launch (SURVEY.md §8(d) per-unit figures x units):
#   walk: headers read (8 or 14 B each at these sizes... counted as the header bytes) + 32 B record
#         + 24 B span written per frame; unmask: 2 x payload + header + 32 B record per frame
CONFIGS = {
    "c1": {"desc": "configs[1] 1 M x 1 KiB BIN, 16 frames/segment", "frames": 1 << 20, "payload": 1 << 30, "hdr": 8},
    "c2": {"desc": "configs[2] 256 Ki mixed 125 B / 64 KiB / 1 MiB, 16 frames/segment", "frames": 262144,
           "payload": 99025807, "hdr": None},
    "head": {"desc": "headline 16 Ki x 64 KiB BIN, 4 frames/segment", "frames": 16384, "payload": 1 << 30, "hdr": 14},
    "c11": {"desc": "configs[1] 1 M x 1 KiB BIN, 1 frame/segment", "frames": 1 << 20, "payload": 1 << 30, "hdr": 8},
    "c4": {"desc": "configs[4] 64 Ki fragmented messages (2..16 fragments of 0..8 KiB), COMPACT", "frames": None,
           "payload": None, "hdr": None},
    "c4i": {"desc": "configs[4]'s batch unmasked in place", "frames": None, "payload": None, "hdr": None},
}
SQ_QUAD = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")   # quad-cycles


def per_kernel(path, counter=None):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if counter and r["Counter_Name"] != counter:
            continue
        agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, _), v in agg.items():
        per[k].append(v)
    return {k: sorted(v)[len(v) // 2] for k, v in per.items()}


def sq_counters(path):
    names = sorted({r["Counter_Name"] for r in csv.DictReader(open(path))})
    return {n: per_kernel(path, n) for n in names}


def main(d):
    out = {"correction": "read = FETCH_SIZE * 1024 * 2 (gfx950 16 B/lane read undercount), write = WRITE_SIZE * 1024",
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 tools/single_loop.py <cfg> 3; median over launches",
           "configs": {}}
    out["sq_note"] = ("SQ_* summed over the dispatch's waves (median dispatch); SQ_WAVE_CYCLES / SQ_WAIT_* / "
                      "SQ_ACTIVE_INST_ANY in quad-cycles (MI355X_MICROARCH.md)")
    for c, meta in CONFIGS.items():
        if not os.path.exists(os.path.join(d, f"fetch_{c}.csv")):
            continue
        f, w = per_kernel(os.path.join(d, f"fetch_{c}.csv")), per_kernel(os.path.join(d, f"write_{c}.csv"))
        sqp = os.path.join(d, f"sq_{c}.csv")
        sq = sq_counters(sqp) if os.path.exists(sqp) else {}
        ks = {}
        for k in f:
            if not k.startswith("wsc::"):
                continue
            ks[k] = {"FETCH_SIZE_KB": f[k], "WRITE_SIZE_KB": w.get(k), "hbm_read_bytes": f[k] * 2048,
                     "hbm_write_bytes": (w.get(k) or 0) * 1024}
            if sq:
                ks[k]["sq"] = {n: v.get(k) for n, v in sq.items()}
                wv = ks[k]["sq"].get("SQ_WAVES")
                if wv:
                    ks[k]["per_wave"] = {n: round(v.get(k, 0) / wv, 1) for n, v in sq.items() if n != "SQ_WAVES"}
        out["configs"][c] = {**meta, "kernels": ks}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
