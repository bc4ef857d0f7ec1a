"""Isolated SpMV timing on C2 (4 rotating copies of A, x, y: no Infinity-Cache reuse)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpu-gmres_amd"))
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

A = M.laplacian_5pt(int(sys.argv[1]) if len(sys.argv) > 1 else 1000)
s = G.Solver()
s.set_matrix(A)
for pre in ("none", "ilu0"):
    getattr(s, "set_precond_" + pre)()
    byt = s.bytes_spmv()
    for nrot in (1, 4):
        ms = s.time_spmv(reps=200, nrot=nrot)
        print(f"layout={'wave' if s.uses_wavefront else 'natural'} nrot={nrot}: {ms*1e3:.2f} us "
              f"{byt/ms/1e6:.0f} GB/s ({byt/ms/1e6/8000:.1%} of 8 TB/s)")
