"""Format GG_MGS_TRACE's raw stderr lines ("mgs_trace i= row= k= t0 t1 t2 t3", s_memrealtime
at 100 MHz) as profiles/r04/r04_mgs_trace.txt's table:
    python tools/diag/mgs_trace_fmt.py gpurun_out/r05_mgs_trace.err > profiles/r05/r05_mgs_trace.txt"""
import re
import sys

rows = {}
i_seen = None
for line in open(sys.argv[1]):
    m = re.match(r"mgs_trace i=(\d+) row=(\d+) k=(\d+) (-?\d+) (-?\d+) (-?\d+) (-?\d+)", line.strip())
    if not m:
        continue
    i, row, k = int(m.group(1)), int(m.group(2)), int(m.group(3))
    i_seen = i
    rows[(row, k)] = [int(m.group(j)) for j in range(4, 8)]
us = lambda t: t / 100.0
print(f"GG_MGS_TRACE=540 (C2, bench --steps 1 --warmup 0): k_arnoldi_persist at inner index i = {i_seen},")
print("device s_memrealtime stamps (100 MHz) per MGS step k: start, h known (all-gather done), partial formed, partial published.")
print("row 0 = unit-block 0, row 1 = the elected reducer of XCD 0.  Times in microseconds.")
print()
print("  k | blk0: gather  axpy+dot  publish  step | reducer: gather  | last-publish(blk0) -> reducer's sum")
ks = sorted(k for (r, k) in rows if r == 0)
g, s = [], []
for k in ks:
    b = rows[(0, k)]
    r = rows.get((1, k))
    nan = float("nan")
    gather = us(b[1] - b[0]) if b[0] > 0 and b[1] > 0 else nan
    axd = us(b[2] - b[1]) if b[1] > 0 and b[2] > 0 else nan      # (the last step, the norm, stamps no partial)
    pub = us(b[3] - b[2]) if b[2] > 0 and b[3] > 0 else nan
    step = us(b[3] - b[0]) if b[0] > 0 and b[3] > 0 else nan
    rg = us(r[1] - r[0]) if r and r[0] > 0 and r[1] > 0 else float("nan")
    prev = rows.get((0, k - 1))
    hop = us(r[1] - prev[3]) if (r and prev and r[1] > 0 and prev[3] > 0) else float("nan")
    if k > 0 and step == step:
        g.append(gather)
        s.append(step)
    print(f"{k:3d} | {gather:7.2f}  {axd:8.2f}  {pub:7.2f}  {step:5.2f} | {rg:6.2f} | {hop:8.2f}")
if g:
    print()
    print(f"mean over steps 1..{ks[-1] - 1}: gather {sum(g) / len(g):.2f} us, step {sum(s) / len(s):.2f} us")
