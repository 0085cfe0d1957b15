"""Summarise tools/pmc_enc.sh: per (kernel, grid) the median dispatch's counters, HBM bytes with the
gfx950 read correction (FETCH_SIZE x 2), and the SQ counters per wave.
usage: python tools/pmc_enc.py <outdir>"""
import collections
import csv
import json
import os
import sys


def load(path):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "wsc::" not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Grid_Size"]))
        agg[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, c, _), v in agg.items():
        per[(k, c)].append(v)
    return {kc: sorted(v)[len(v) // 2] for kc, v in per.items()}


d = sys.argv[1]
vals = {}
for p in ("fetch", "write", "sq"):
    f = os.path.join(d, p + ".csv")
    if os.path.exists(f):
        vals.update(load(f))
res = {}
for (k, c), v in sorted(vals.items()):
    res.setdefault(f"{k[0]} grid {k[1]}", {})[c] = v
for name, r in res.items():
    if "FETCH_SIZE" in r:
        r["hbm_read_bytes"] = r["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in r:
        r["hbm_write_bytes"] = r["WRITE_SIZE"] * 1024
    w = r.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in r:
                r[c + "_per_wave"] = round(r[c] / w, 1)
print(json.dumps(res, indent=1))
