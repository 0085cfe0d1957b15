"""Split a rocprofv3 kernel trace by (kernel, grid size).

`rocprofv3 --kernel-trace --stats` averages every launch of a kernel together; bench.py launches
k_unmask for the headline batch and for the other configs, so the stats average mixes sizes. This
groups the per-dispatch rows of `*_kernel_trace.csv` by kernel name and grid size and prints the
count / average / median / min / max duration of each group, so the headline launch's rocprof
duration can be compared with the hipEvent time bench.py reports.

usage: python tools/rocprof_split.py <dir-or-kernel_trace.csv> [--match SUBSTR] [--out FILE]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def find_trace(path):
    if os.path.isfile(path):
        return [path]
    return sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="wsc::")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    groups = {}
    for f in find_trace(a.path):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if a.match and a.match not in name:
                    continue
                grid = int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0)
                wg = int(row.get("Workgroup_Size_X") or row.get("Workgroup_Size") or 0)
                dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                groups.setdefault((short(name), grid, wg), []).append(dur)
    rows = []
    for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        rows.append({"kernel": name, "grid_x": grid, "wg_x": wg, "calls": len(d),
                     "avg_us": round(statistics.mean(d) / 1e3, 2),
                     "median_us": round(statistics.median(d) / 1e3, 2),
                     "min_us": round(min(d) / 1e3, 2), "max_us": round(max(d) / 1e3, 2)})
    for r in rows:
        print(f'{r["kernel"]:<40} grid {r["grid_x"]:>9} wg {r["wg_x"]:>4} calls {r["calls"]:>5} '
              f'avg {r["avg_us"]:>9.2f} us  median {r["median_us"]:>9.2f}  min {r["min_us"]:>9.2f}  max {r["max_us"]:>9.2f}')
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
