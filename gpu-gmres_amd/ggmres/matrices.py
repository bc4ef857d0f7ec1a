"""Synthetic and fixture matrices for the GMRES path.

Configs:
  C1  100x100 5-pt Dirichlet Laplacian (diag 4, off -1), natural order, n=10,000
  C2  1000x1000 5-pt, n=1,000,000, nnz=4,996,000
  C3  circuit5M stand-in (the SuiteSparse file is not available offline):
      seeded power-law CSR with circuit5M's n and nnz (power_law)
  C4  7-pt 3D thermal grid, kx=ky=1, kz=10, diag = sum|off| + 1e-3
  C5  A = G + C/h with C = c*I

All matrices are scipy.sparse CSR, float64 values, int32 indices sorted per row.
"""
import numpy as np
import scipy.sparse as sp


def _finish(A):
    A = sp.csr_matrix(A)
    A.sum_duplicates()
    A.sort_indices()
    A.indptr = A.indptr.astype(np.int32)
    A.indices = A.indices.astype(np.int32)
    A.data = A.data.astype(np.float64)
    return A


def laplacian_5pt(nx, ny=None, diag=4.0, off=-1.0):
    """2D 5-point stencil, natural row-major order (row r = j*nx + i)."""
    ny = nx if ny is None else ny
    n = nx * ny
    r = np.arange(n, dtype=np.int64)
    i = r % nx
    j = r // nx
    rows = [r]
    cols = [r]
    vals = [np.full(n, diag)]
    for di, dj in ((-1, 0), (1, 0), (0, -1), (0, 1)):
        ok = (i + di >= 0) & (i + di < nx) & (j + dj >= 0) & (j + dj < ny)
        rows.append(r[ok])
        cols.append(r[ok] + di + dj * nx)
        vals.append(np.full(int(ok.sum()), off))
    A = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n, n))
    return _finish(A)


def grid_7pt(nx, ny=None, nz=None, kx=1.0, ky=1.0, kz=10.0, shift=1e-3, upwind=0.0,
             const_diag=None):
    """3D 7-point thermal grid (C4).  Off-diagonals -k per direction (x gets an
    optional +-upwind asymmetry); diagonal = sum|off| + shift (convective
    boundary), or const_diag everywhere (Dirichlet Laplacian, e.g. 7)."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    n = nx * ny * nz
    r = np.arange(n, dtype=np.int64)
    i = r % nx
    j = (r // nx) % ny
    k = r // (nx * ny)
    rows, cols, vals = [], [], []
    dsum = np.zeros(n)
    for (di, dj, dk, w) in ((-1, 0, 0, kx * (1 + upwind)), (1, 0, 0, kx * (1 - upwind)),
                            (0, -1, 0, ky), (0, 1, 0, ky), (0, 0, -1, kz), (0, 0, 1, kz)):
        ok = ((i + di >= 0) & (i + di < nx) & (j + dj >= 0) & (j + dj < ny)
              & (k + dk >= 0) & (k + dk < nz))
        rows.append(r[ok])
        cols.append(r[ok] + di + dj * nx + dk * nx * ny)
        vals.append(np.full(int(ok.sum()), -w))
        dsum[ok] += w
    rows.append(r)
    cols.append(r)
    vals.append(dsum + shift if const_diag is None else np.full(n, float(const_diag)))
    A = sp.coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n, n))
    return _finish(A)


def transient(G, c=1e-3, h=1e-2):
    """A = G + C/h with C = c*I (C5, backward Euler)."""
    n = G.shape[0]
    return _finish(G + sp.identity(n, format="csr") * (c / h))


def pulse_sources(n, frac=0.01, h=1e-2, seed=20261015):
    """C5 sources: a seeded 1 % of the nodes each carry a PULSE
    current, vlo 0, vhi 1e-3, td 0, tr = tf = 10 h, tw = 100 h, period 400 h.
    Returns (src_node int32[nsrc], pulses float64[nsrc, 7] as
    {vlo, vhi, td, tr, tf, tw, tp})."""
    rng = np.random.default_rng(seed)
    nsrc = max(1, int(round(frac * n)))
    nodes = np.sort(rng.choice(n, size=nsrc, replace=False)).astype(np.int32)
    q = np.array([0.0, 1e-3, 0.0, 10 * h, 10 * h, 100 * h, 400 * h])
    return nodes, np.tile(q, (nsrc, 1))


def read_mtx(path):
    import scipy.io
    return _finish(scipy.io.mmread(path))


def _fortran_width(fmt):
    """'(10I8)' -> (10, 8); '(5E16.8)' -> (5, 16); '(4D20.12)' -> (4, 20)."""
    import re
    m = re.search(r"(\d+)\s*[IEDFGiedfg]\s*(\d+)", fmt.replace("1P", "").replace("1p", ""))
    return int(m.group(1)), int(m.group(2))


def read_rua(path):
    """Harwell-Boeing real unsymmetric assembled matrix (e.g. sherman1.rua).
    Columns are stored compressed (CSC); right-hand-side blocks are ignored."""
    with open(path) as f:
        lines = f.read().split("\n")
    counts = lines[1]
    ptrcrd, indcrd, valcrd = int(counts[14:28]), int(counts[28:42]), int(counts[42:56])
    mxtype = lines[2][:3].upper()
    if mxtype != "RUA":
        raise ValueError(f"{path}: only RUA supported, got {mxtype}")
    nrow, ncol, nnz = int(lines[2][14:28]), int(lines[2][28:42]), int(lines[2][42:56])
    fmts = lines[3]
    pw = _fortran_width(fmts[0:16])[1]
    iw = _fortran_width(fmts[16:32])[1]
    vw = _fortran_width(fmts[32:52])[1]
    rhscrd = counts[56:70].strip()
    start = 4 + (1 if rhscrd and int(rhscrd) > 0 else 0)

    def fields(block, w):
        out = []
        for ln in block:
            ln = ln.rstrip()
            out.extend(ln[k:k + w] for k in range(0, len(ln), w))
        return [t for t in out if t.strip()]

    ptr = np.array([int(t) for t in fields(lines[start:start + ptrcrd], pw)], np.int64) - 1
    start += ptrcrd
    ind = np.array([int(t) for t in fields(lines[start:start + indcrd], iw)], np.int64) - 1
    start += indcrd
    val = np.array([float(t.replace("D", "E").replace("d", "e"))
                    for t in fields(lines[start:start + valcrd], vw)])
    assert len(ptr) == ncol + 1 and len(ind) == nnz and len(val) == nnz
    A = sp.csc_matrix((val, ind, ptr), shape=(nrow, ncol))
    return _finish(A.tocsr())


def power_law(n=5_558_326, nnz=59_524_291, alpha=1.5, cap=100_000, seed=20261015):
    """Synthetic stand-in for C3: off-diagonal counts per row
    ~ Zipf(alpha) clipped to [1, cap], rescaled (stochastic rounding) so the
    matrix holds about `nnz` entries; columns uniform; values -U(0,1); the
    diagonal is the row's sum of |off| + 1 (strictly diagonally dominant).
    Heavy-tailed rows (a few thousand entries) exercise the long-row path."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k = np.minimum(rng.zipf(alpha, n), cap).astype(np.float64)
    k *= (nnz - n) / k.sum()
    k = np.floor(k + rng.random(n)).astype(np.int64)
    k = np.minimum(k, n - 1)
    tot = int(k.sum())
    rows = np.repeat(np.arange(n, dtype=np.int64), k)
    cols = rng.integers(0, n - 1, tot, dtype=np.int64)
    cols += cols >= rows                       # skip the diagonal
    vals = -rng.random(tot)
    A = sp.coo_matrix((vals, (rows, cols)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    d = np.asarray(abs(A).sum(axis=1)).ravel() + 1.0
    return _finish(A + sp.diags(d))


def rhs_ones(A):
    """b = A * 1 (the x_exact = 1 idiom, src/mna_solve_gmres.cpp:302-303)."""
    return A @ np.ones(A.shape[0])


def rhs_uniform(n, seed=20261015):
    """b ~ U[0,1) from PCG64(seed)."""
    return np.random.Generator(np.random.PCG64(seed)).random(n)


def pg_netlist(path, nx, ny, pad_stride=50, isrc_frac=0.01, seed=20261015):
    """Write a synthetic IBM-power-grid-style flat SPICE netlist (the reference
    driver's input, src/parser.cpp:69-272, 1904-2886; read back by
    ggmres.host.Netlist = gg_host_read_netlist): an nx x ny resistor mesh (one
    metal layer, 0.05-0.5 ohm segments), a 10-90 fF decoupling capacitor from
    every node to ground (listed FIRST, so the MNA numbers the grid nodes in
    row-major order), load currents (PULSE, 0 -> 1-5 mA) at a seeded
    `isrc_frac` of the nodes, and a VDD pad every `pad_stride` nodes in both
    directions: a 10 mOhm package resistor to a pad node held at 1.8 V by a
    voltage source (MNA: one branch-current row each, zero diagonal).
    Returns (n_grid, n_pads)."""
    rng = np.random.default_rng(seed)
    nm = lambda j, i: f"n{j}_{i}"
    out = ["* synthetic IBM-PG-style power grid", ".tran 10p 1n"]
    cap = rng.integers(10, 91, (ny, nx))
    for j in range(ny):
        out.extend(f"C{j}_{i} {nm(j, i)} 0 {cap[j, i]}f" for i in range(nx))
    rh = rng.uniform(0.05, 0.5, (ny, nx))
    rv = rng.uniform(0.05, 0.5, (ny, nx))
    for j in range(ny):
        for i in range(nx):
            if i + 1 < nx:
                out.append(f"R{j}_{i}h {nm(j, i)} {nm(j, i + 1)} {rh[j, i]:.5f}")
            if j + 1 < ny:
                out.append(f"R{j}_{i}v {nm(j, i)} {nm(j + 1, i)} {rv[j, i]:.5f}")
    n = nx * ny
    loads = np.sort(rng.choice(n, size=max(1, int(round(isrc_frac * n))), replace=False))
    amp = rng.uniform(1.0, 5.0, loads.size)
    for k, (r, a) in enumerate(zip(loads, amp)):
        out.append(f"I{k} {nm(r // nx, r % nx)} 0 0 PULSE(0, {a:.3f}m, 50p, 20p, 20p, 200p, 500p)")
    npad = 0
    for j in range(pad_stride // 2, ny, pad_stride):
        for i in range(pad_stride // 2, nx, pad_stride):
            out.append(f"Rp{npad} {nm(j, i)} X{npad} 10m")
            out.append(f"V{npad} X{npad} 0 1.8")
            npad += 1
    out.append(f".print tran v({nm(0, 0)}) v({nm(ny // 2, nx // 2)})")
    out.append(".end")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    return n, npad


def mna_pivot_order(n_grid, n_pads, n):
    """Row / column permutations that give an MNA system with voltage-source
    branch rows (zero diagonal) a nonzero diagonal for ILU(0) -- the pivoting
    ILU++'s factorization does for the reference's PG path
    (src/mna_solve_gpu_gmres.cpp:316-474).  Unknowns (gg_host_read_netlist):
    [grid nodes | pad nodes X_k | branch currents I_k]; the branch row I_k
    (V_{X_k} = V) has its only entry in column X_k, X_k's KCL row has +1 in
    column I_k.  Returned as (prow, pcol) in the split engine's convention
    (B = P_r A P_c: B row i = A row prow[i], B column pcol[c] = A column c):
    the tail (pad and branch unknowns) FIRST -- B rows [I_k ..., X_k ..., grid],
    B columns [X_k ..., I_k ..., grid] -- so the grid block keeps its 5-point
    pattern, its rows referencing the tail only in columns left of the grid."""
    assert n == n_grid + 2 * n_pads
    X = np.arange(n_grid, n_grid + n_pads)
    I = np.arange(n_grid + n_pads, n)
    grid = np.arange(n_grid)
    prow = np.concatenate([I, X, grid]).astype(np.int32)
    colorder = np.concatenate([X, I, grid])          # B column c = A column colorder[c]
    pcol = np.empty(n, np.int32)
    pcol[colorder] = np.arange(n, dtype=np.int32)
    return prow, pcol
