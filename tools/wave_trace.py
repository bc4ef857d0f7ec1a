"""Diagnostics: per-band batch timing of the wavefront triangular solves on C2.

python tools/wave_trace.py [--grid 1000]  (GPU) -> band start lags, batch times,
the compute wave's per-batch phase cycles and the hand-off latency (writer
publish -> consumer boundary wave sees it) for the L and U solves."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-gmres_amd"))
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=1000)
ap.add_argument("--division", choices=["exact", "rcp", "fma"], default="fma")
args = ap.parse_args()
A = M.laplacian_5pt(args.grid)
s = G.Solver()
s.set_matrix(A)
s.set_precond_ilu0()
s.set_division({"exact": G.DIV_EXACT, "rcp": G.DIV_RCP, "fma": G.DIV_FMA}[args.division])
print("division", args.division, "kernels", s.trsv_kernel(0), "/", s.trsv_kernel(1))
b = np.ones(A.shape[0])
s.precond_apply(0, b)
print("precond apply avg ms", s.time_precond(20))
for which in (0, 1):
    for rep in range(2):
        raw = s.trace_precond(which)
    nb = raw.shape[0]
    nbt = (raw.shape[1] - 8) // 3
    KB = (args.grid + 63 + 31) // 32 * 32 // nbt      # steps per batch
    t0 = raw[:, 0].min()
    comp = (raw[:, :nbt + 1] - t0) * 0.01           # us
    ph = raw[:, nbt + 1:nbt + 5].astype(np.float64)
    bw = raw[:, nbt + 5:nbt + 7].astype(np.float64)
    pub = (raw[:, nbt + 8:2 * nbt + 8] - t0) * 0.01
    seen = (raw[:, 2 * nbt + 8:3 * nbt + 8] - t0) * 0.01
    start, end = comp[:, 0], comp[:, -1]
    d = np.diff(comp, axis=1)
    print(f"{'LU'[which]}: total {end.max():.1f} us, nbands {nb}, nbatch {nbt}")
    print("  start lag (us):", np.round(np.diff(start), 2).tolist())
    print("  batch us median per band:", np.round(np.median(d, axis=1), 3).tolist())
    print("  phase cycles/batch [barrier, top->s0, s0->last, last->end] (mean over bands):",
          np.round(ph.mean(axis=0) / nbt, 0).tolist())
    print("  boundary retries/batch per band:", np.round(bw[:, 0] / nbt, 2).tolist())
    # hand-off: consumer batch bi needs producer steps up to KB*bi+KB-1+63 -> producer batch
    lat, ahead = [], []
    for c in range(nb):
        p = c - 1 if which == 0 else c + 1
        if p < 0 or p >= nb:
            continue
        for bi in range(2, nbt - 10):
            k = (KB * bi + KB - 1 + 63) // KB
            if k < nbt:
                lat.append(seen[c, bi] - pub[p, k])
                ahead.append(comp[c, bi] - seen[c, bi])
    lat = np.array(lat)
    print(f"  publish -> seen latency us: median {np.median(lat):.2f} p10 {np.percentile(lat, 10):.2f} "
          f"p90 {np.percentile(lat, 90):.2f}")
    print(f"  seen -> consumer batch start us: median {np.median(ahead):.2f}")
    wr = []
    for c in range(nb):
        for k in range(1, nbt - 1):
            wr.append(pub[c, k] - comp[c, k])
    print(f"  producer batch start -> publish us: median {np.median(wr):.2f}")
