"""Median gap before each kernel, per (previous kernel -> kernel) pair on the same queue, and
median durations: python tools/kt_gaps.py trace.csv"""
import collections
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
byq = collections.defaultdict(list)
for r in rows:
    byq[r["Queue_Id"]].append(r)
gaps, durs = collections.defaultdict(list), collections.defaultdict(list)
short = lambda n: n.split("(")[0].replace("void ", "").replace("wsc::", "")[:32]
for q, rs in byq.items():
    for a, b in zip(rs, rs[1:]):
        gaps[(q, short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
    for r in rs:
        durs[(q, short(r["Kernel_Name"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(durs.items()):
    print(f"dur q{k[0]} {k[1]:34s} n={len(v):4d} med {statistics.median(v):9.1f} us")
for k, v in sorted(gaps.items()):
    if len(v) >= 3:
        print(f"gap q{k[0]} {k[1]:34s} -> {k[2]:34s} n={len(v):4d} med {statistics.median(v):8.1f} us")
