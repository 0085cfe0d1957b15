"""Per-step breakdown of a pipelined bench kernel trace (rocprofv3 --kernel-trace csv): for each
burst of walks on the walk queue, the unmask durations and the gaps between consecutive unmasks."""
import csv
import statistics
import sys


def main(path, walk_q=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    qs = {}
    for r in rows:
        if "walk" in r["Kernel_Name"]:
            qs[r["Queue_Id"]] = qs.get(r["Queue_Id"], 0) + 1
    # the walk queue of the split pipeline: the queue with walks that is not the one with unmasks too
    unq = {r["Queue_Id"] for r in rows if "unmask" in r["Kernel_Name"]}
    wq = walk_q or next((q for q in qs if q not in unq), None)
    walks = [r for r in rows if r["Queue_Id"] == wq]
    if not walks:
        print("no split pipeline in", path)
        return
    bursts, cur = [], [walks[0]]
    for a, b in zip(walks, walks[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 2_000_000:
            bursts.append(cur)
            cur = []
        cur.append(b)
    bursts.append(cur)
    for bw in bursts:
        lo, hi = int(bw[0]["Start_Timestamp"]), int(bw[-1]["End_Timestamp"]) + 400_000
        um = [r for r in rows if "unmask" in r["Kernel_Name"] and lo <= int(r["Start_Timestamp"]) <= hi]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in um]
        g = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(um, um[1:])]
        span = (int(um[-1]["End_Timestamp"]) - int(um[0]["Start_Timestamp"])) / 1e3
        other = [r["Kernel_Name"][:20] for r in rows if lo <= int(r["Start_Timestamp"]) <= hi
                 and r["Queue_Id"] != wq and "unmask" not in r["Kernel_Name"]]
        print(f"walks {len(bw)} unmasks {len(um)} dur med {statistics.median(d):.1f} mean {statistics.mean(d):.1f} "
              f"gap med {statistics.median(g):.2f} mean {statistics.mean(g):.2f} step {span / len(um):.1f} us; "
              f"other kernels on the unmask queue: {len(other)}; gaps {[round(x, 1) for x in g[:10]]}")


if __name__ == "__main__":
    main(sys.argv[1])
