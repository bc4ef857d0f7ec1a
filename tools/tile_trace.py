"""Diagnostics: tile schedule of the 3D tile wavefront triangular solves (C4).

python tools/tile_trace.py [--grid 216]  (GPU) -> per solve: total time, tile
duration, start lag of a tile behind its line / plane source, batch-0 time,
boundary-wave retries, and how far the workgroups' tile lists serialise."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-gmres_amd"))
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=216)
ap.add_argument("--save", default=None, help="write the raw traces (L, U) to this .npz")
args = ap.parse_args()
n1 = args.grid
A = M.grid_7pt(n1)
s = G.Solver()
s.set_matrix(A)
s.set_precond_ilu0()
b = np.ones(A.shape[0])
s.precond_apply(0, b)
print("precond apply avg ms", s.time_precond(10))
NJ, NK = (n1 + 7) // 8, (n1 + 7) // 8
raws = {}
for which in (0, 1):
    for rep in range(2):
        raw = s.trace_tiles(which)
    raws["LU"[which]] = raw
    t0 = raw[:, 6].min()
    st = (raw[:, 0] - t0) * 0.01
    en = (raw[:, 1] - t0) * 0.01
    b0 = (raw[:, 5] - raw[:, 0]) * 0.01
    ld = (raw[:, 6] - t0) * 0.01
    wg = raw[:, 2]
    S = st.reshape(NK, NJ)
    dur = en - st
    print(f"{'LU'[which]}: total {en.max():.1f} us, tiles {len(st)}, workgroups {len(np.unique(wg))}")
    print(f"  tile duration us: median {np.median(dur):.2f} p10 {np.percentile(dur, 10):.2f} "
          f"p90 {np.percentile(dur, 90):.2f}; batch 0 median {np.median(b0):.2f}")
    if which == 0:
        lj = np.diff(S, axis=1)
        lk = np.diff(S, axis=0)
    else:
        lj = -np.diff(S, axis=1)
        lk = -np.diff(S, axis=0)
    print(f"  start lag behind line source us: median {np.median(lj):.2f} p90 {np.percentile(lj, 90):.2f}")
    print(f"  start lag behind plane source us: median {np.median(lk):.2f} p90 {np.percentile(lk, 90):.2f}")
    print(f"  loader start -> compute start us: median {np.median(st - ld):.2f} p90 {np.percentile(st - ld, 90):.2f}")
    print(f"  boundary retries per tile: median {np.median(raw[:, 3]):.0f}, retry cycles median {np.median(raw[:, 4]):.0f}")
    # how many tiles run at once (sampled)
    ts = np.linspace(0, en.max(), 50)
    conc = [int(((st <= t) & (en > t)).sum()) for t in ts]
    print("  concurrently running tiles over time:", conc)
    # per batch: hand-off latency (the later source's publication -> values
    # seen), seen -> compute batch start, and the batch time
    nbt = (raw.shape[1] - 8) // 5
    KB = 8
    comp = (raw[:, 8:8 + nbt] - t0) * 0.01
    pub = (raw[:, 8 + nbt:8 + 2 * nbt] - t0) * 0.01
    seen = (raw[:, 8 + 2 * nbt:8 + 3 * nbt] - t0) * 0.01
    lat, ahead, which_src, srcgap = [], [], [], []
    for q in range(len(st)):
        J, K = q % NJ, q // NJ
        sj = (J - 1 if which == 0 else J + 1)
        sk = (K - 1 if which == 0 else K + 1)
        for bi in range(1, nbt - 3):
            need = []
            if 0 <= sk < NK:
                kb = (KB * bi + KB - 1 + 7) // KB     # plane granules: step t + 7 (skew a + c)
                if kb < nbt:
                    need.append(pub[sk * NJ + J, kb])
            if 0 <= sj < NJ:
                jb = (KB * bi + KB - 1 + 7) // KB
                if jb < nbt:
                    need.append(pub[K * NJ + sj, jb])
            if len(need) == 2:
                which_src.append(int(need[1] > need[0]))
                srcgap.append(abs(need[1] - need[0]))
            if need:
                lat.append(seen[q, bi] - max(need))
                ahead.append(comp[q, bi] - seen[q, bi])
    lat, ahead = np.array(lat), np.array(ahead)
    print(f"  publish -> seen us: median {np.median(lat):.2f} p10 {np.percentile(lat, 10):.2f} p90 {np.percentile(lat, 90):.2f}")
    print(f"  seen -> batch start us: median {np.median(ahead):.2f} p90 {np.percentile(ahead, 90):.2f}")
    if which_src:
        print(f"  line source is the later one in {100 * np.mean(which_src):.0f} % of batches, "
              f"gap median {np.median(srcgap):.2f} us")
    bt = np.diff(comp, axis=1)
    print(f"  batch time us: median {np.median(bt):.2f} p10 {np.percentile(bt, 10):.2f}")
    pubd = pub - comp
    print(f"  batch start -> published us: median {np.median(pubd):.2f}")
    land = (raw[:, 8 + 3 * nbt:8 + 4 * nbt] - t0) * 0.01
    cend = (raw[:, 8 + 4 * nbt:8 + 5 * nbt] - t0) * 0.01
    cd = cend - comp
    print(f"  compute of a batch us: median {np.median(cd):.2f} p10 {np.percentile(cd, 10):.2f} p90 {np.percentile(cd, 90):.2f}")
    print(f"  compute end -> published us: median {np.median(pub - cend):.2f}")
    # what the batch start waited for last: landed, seen, or the previous batch's compute
    last = np.argmax(np.stack([land[:, 1:], seen[:, 1:], cend[:, :-1]]), axis=0)
    print("  batch start gated by [loader, boundary, compute] (fraction):",
          np.round(np.bincount(last.ravel(), minlength=3) / last.size, 2).tolist())
    print(f"  loader landed -> batch start us: median {np.median(comp[:, 1:] - land[:, 1:]):.2f}; "
          f"landed minus prev compute end median {np.median(land[:, 1:] - cend[:, :-1]):.2f}")
    # first row of tiles (K = 0 forward / last backward): line-direction chain
    kk = 0 if which == 0 else NK - 1
    print("  starts along J at K=%d:" % kk, np.round(S[kk], 1).tolist())
    jj = 0 if which == 0 else NJ - 1
    print("  starts along K at J=%d (every 4th):" % jj, np.round(S[::4, jj], 1).tolist())

if args.save:
    np.savez_compressed(args.save, NJ=NJ, NK=NK, **raws)
