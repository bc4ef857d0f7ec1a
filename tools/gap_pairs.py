"""Idle gaps between consecutive kernels by (previous, next) kernel pair, from a
rocprofv3 kernel trace: python tools/gap_pairs.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("gg::", "")
    return n.split("(")[0][:40]


gap = collections.defaultdict(list)
dur = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gap[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
for r in rows:
    dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
busy = sum(sum(v) for v in dur.values())
print(f"span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, idle {100 * (1 - busy / span):.1f} %")
for k in sorted(gap, key=lambda k: -sum(gap[k]))[:14]:
    g = sorted(gap[k])
    print(f"{k[0]:40s} -> {k[1]:40s} n={len(g):6d} med {g[len(g) // 2] / 1e3:6.2f} us  total {sum(g) / 1e3:9.1f} us")
for k in sorted(dur, key=lambda k: -sum(dur[k]))[:8]:
    d = sorted(dur[k])
    print(f"{k:40s} n={len(d):6d} med {d[len(d) // 2] / 1e3:7.2f} us")
