"""Diagnostics: per-band batch timing of the wavefront triangular solves on C2.

python tools/wave_trace.py [--grid 1000]  (GPU) -> band start lags, batch times
and the compute wave's per-batch phase cycles for the L and U solves."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-gmres_amd"))
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=1000)
args = ap.parse_args()
A = M.laplacian_5pt(args.grid)
s = G.Solver()
s.set_matrix(A)
s.set_precond_ilu0()
b = np.ones(A.shape[0])
s.precond_apply(0, b)
print("precond apply avg ms", s.time_precond(20))
for which in (0, 1):
    for rep in range(2):
        raw = s.trace_precond(which)
    ph = raw[:, -4:].astype(np.float64)
    tr = raw[:, :-4].astype(np.float64) * 0.01   # us
    tr -= tr[:, 0].min()
    nb, nbt1 = tr.shape
    nbt = nbt1 - 1
    start, end = tr[:, 0], tr[:, -1]
    d = np.diff(tr, axis=1)
    print(f"{'LU'[which]}: total {end.max():.1f} us, nbands {nb}, nbatch {nbt}")
    print("  start lag (us):", np.round(np.diff(start), 2).tolist())
    print("  batch us median per band:", np.round(np.median(d, axis=1), 3).tolist())
    print("  phase cycles/batch [barrier, top->s0, s0->last, last->end] (mean over bands):",
          np.round(ph.mean(axis=0) / nbt, 0).tolist())
    first = 0 if which == 0 else nb - 1
    print("  free-running band phases:", np.round(ph[first] / nbt, 0).tolist())
