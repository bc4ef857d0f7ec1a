import sys, os
sys.path.insert(0, '/root/repo/gpu-gmres_amd'); sys.path.insert(0, '/root/repo')
import numpy as np
import scipy.sparse as sp
import ggmres as G, oracle as O
from ggmres import matrices as M
s = G.Solver()
for dims in [(20,20,3),(10,20,3),(10,17,3),(10,16,3),(10,15,3)]:
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz, upwind=0.1)
    n = A.shape[0]
    L, U = O.ilu0(A)
    I = sp.identity(n, format="csr")
    s.set_matrix(A)
    s.set_precond_lu((n, L.rp, L.ci, L.v), I)
    y = np.random.default_rng(8).standard_normal(n)
    z = s.precond_apply(G.APPLY_MINV, y)
    Id = O.csr(I)
    ref = O.lusolve(L, Id, y)
    bad = np.nonzero(z != ref)[0]
    print(dims, "L only", s.uses_wavefront, len(bad), flush=True)
    if len(bad):
        q = bad[0]
        print("  first bad (i,j,k):", int(q % nx), int((q // nx) % ny), int(q // (nx*ny)), z[q], ref[q])
        per = [int(((bad // (nx*ny)) == k).sum()) for k in range(nz)]
        print("  bad per plane:", per)
s.close()
