"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py into per-launch HBM bytes of the
unmask kernel, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KB) reads 1/2 of the
bytes of a wide (16 B/lane) streaming read on gfx950 -> x2; WRITE_SIZE (KB) is exact for 16 B/lane
streaming stores.  Writes profiles/pmc_traffic.json (read by bench.py for roofline.traffic)."""
import csv
import json
import sys

import numpy as np


def per_kernel(path, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return vals


def main(fetch_csv, write_csv, out, frames, frame_bytes):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    res = {"frames": frames, "frame_bytes": frame_bytes, "kernels": {}}
    for name in sorted(set(f) | set(w)):
        if "wsc::" not in name:
            continue
        fk = float(np.median(f.get(name, [0])))
        wk = float(np.median(w.get(name, [0])))
        short = name.split("(")[0].replace("void ", "")
        res["kernels"][short] = {"FETCH_SIZE_KB_median": fk, "WRITE_SIZE_KB_median": wk,
                                 "hbm_read_bytes": fk * 1024 * 2, "hbm_write_bytes": wk * 1024,
                                 "launches": len(f.get(name, []))}
    um = sorted((k for k in res["kernels"] if "k_unmask" in k), key=lambda k: -res["kernels"][k]["launches"])
    if um:   # the headline's unmask: the variant launched most (the pipelined binary kernel)
        res["unmask_kernel"] = um[0]
        k = res["kernels"][um[0]]
        res["unmask_hbm_bytes_per_launch"] = k["hbm_read_bytes"] + k["hbm_write_bytes"]
    hdr = 14 if frame_bytes > 65535 else (8 if frame_bytes > 125 else 6)
    res["unmask_alg_bytes_per_launch"] = frames * (2 * frame_bytes + hdr + 32)
    res["correction"] = "read = FETCH_SIZE*1024*2 (gfx950 wide-read undercount), write = WRITE_SIZE*1024"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
