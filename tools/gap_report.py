"""Per-kernel duration and the idle gap before each launch, from a rocprofv3
kernel trace: python tools/gap_report.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gap = collections.defaultdict(list)
dur = collections.defaultdict(list)
prev = None
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0][-48:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[n].append(e - s)
    if prev is not None:
        gap[n].append(s - prev)
    prev = e
for n in sorted(dur, key=lambda k: -sum(dur[k])):
    g = sorted(gap[n])
    print(f"{n:48s} n={len(dur[n]):6d} dur={sum(dur[n]) / len(dur[n]) / 1e3:8.2f}us "
          f"gap_med={(g[len(g) // 2] if g else 0) / 1e3:6.2f}us")
