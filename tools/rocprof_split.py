"""Split a rocprofv3 kernel trace by (kernel, grid size).

`rocprofv3 --kernel-trace --stats` averages every launch of a kernel together; bench.py launches
k_unmask for the headline batch and for the other configs, so the stats average mixes sizes. This
groups the per-dispatch rows of `*_kernel_trace.csv` by kernel name and grid size and prints the
count / average / median / min / max duration of each group, so the headline launch's rocprof
duration can be compared with the hipEvent time bench.py reports.

Reads CSV traces (`--output-format csv`) or the rocpd SQLite database ROCm 7's rocprofv3 writes by
default (`*_results.db`, view `kernels`); `--stats FILE` also writes a kernel-stats CSV in the
layout of rocprofv3's `kernel_stats.csv` (from the database).

usage: python tools/rocprof_split.py <dir-or-trace> [--match SUBSTR] [--out FILE] [--stats FILE]
"""
import argparse
import csv
import glob
import json
import os
import sqlite3
import statistics


def find_trace(path):
    if os.path.isfile(path):
        return [path]
    found = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))
    return found or sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))


def dispatches(f):
    """(kernel name, grid_x, workgroup_x, duration ns) per dispatch"""
    if f.endswith(".db"):
        con = sqlite3.connect(f)
        for name, grid, wg, dur in con.execute("select name, grid_x, workgroup_x, duration from kernels"):
            yield name, int(grid), int(wg), int(dur)
        con.close()
        return
    with open(f, newline="") as fh:
        for row in csv.DictReader(fh):
            yield (row.get("Kernel_Name", ""), int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0),
                   int(row.get("Workgroup_Size_X") or row.get("Workgroup_Size") or 0),
                   int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))


def write_stats(files, out):
    per = {}
    for f in files:
        for name, _, _, dur in dispatches(f):
            per.setdefault(name, []).append(dur)
    total = sum(sum(d) for d in per.values()) or 1
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), f"{statistics.mean(d):.6f}", f"{100 * sum(d) / total:.2f}", min(d), max(d),
                        f"{statistics.pstdev(d):.6f}"])


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="wsc::")
    ap.add_argument("--out", default="")
    ap.add_argument("--stats", default="")
    a = ap.parse_args()
    groups = {}
    files = find_trace(a.path)
    if a.stats:
        write_stats(files, a.stats)
    for f in files:
        for name, grid, wg, dur in dispatches(f):
            if a.match and a.match not in name:
                continue
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
