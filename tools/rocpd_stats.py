"""Kernel summary from a rocprofv3 rocpd database (run_results.db): per kernel
name the launches, total / average duration and share of GPU time, and the
same split by grid size (gated launches are short).  Usage:
    python tools/rocpd_stats.py DB [--by-grid] [--top N] [--csv OUT]"""
import argparse
import collections
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--top", type=int, default=25)
    p.add_argument("--csv")
    p.add_argument("--gated-us", type=float, default=0.0,
                   help="also count launches shorter than this (a gated launch's dispatch)")
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    names = dict(c.execute("select id, display_name from rocpd_info_kernel_symbol"))
    agg = collections.defaultdict(lambda: [0, 0.0, 0, 0.0])
    total = 0.0
    for kid, st, en in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        d = (en - st) * 1e-3
        r = agg[names.get(kid, str(kid))]
        r[0] += 1
        r[1] += d
        if d < a.gated_us:
            r[2] += 1
            r[3] += d
        total += d
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"{'kernel':<90} {'calls':>8} {'total_ms':>10} {'avg_us':>9} {'pct':>6} {'short':>7} {'short_ms':>9}")
    for k, (n, t, ns, ts) in rows[:a.top]:
        print(f"{k[:90]:<90} {n:>8} {t/1e3:>10.3f} {t/n:>9.2f} {100*t/total:>6.2f} {ns:>7} {ts/1e3:>9.3f}")
    print(f"total GPU time {total/1e3:.3f} ms over {sum(v[0] for v in agg.values())} launches")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("Name,Calls,TotalDurationNs,AverageNs,Percentage\n")
            for k, (n, t, _, _) in rows:
                f.write(f"\"{k}\",{n},{int(t*1e3)},{t*1e3/n:.1f},{100*t/total:.4f}\n")


if __name__ == "__main__":
    main()
