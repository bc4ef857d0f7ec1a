"""Shared test helpers: synthetic split (ILU++/PG) preconditioners, comparisons."""
import numpy as np
import scipy.sparse as sp

import oracle as O


def csr_sp(T):
    """oracle CSR tuple -> scipy csr"""
    return sp.csr_matrix((T.v, T.ci, T.rp), shape=(T.n, T.n))


def make_split(A, seed=7, identity_perm=False, perm=None):
    """Synthetic PG split preconditioner for A.

    With pcol = prow^-1, B = P_r D_l^-1 A D_r^-1 P_c is a symmetric permutation
    of a scaled A; B ~= Lt Ut (oracle ILU(0)); L = Lt D1 (non-unit, diag last),
    U = M D1^-1 Ut (diag first) so that Ml A Mr = L^-1 B U^-1 M ~= I.
    identity_perm: P_r = P_c = I (the factors of a grid stay grid-shaped: the
    split engine's 2D wavefront path).  perm: explicit (prow, pcol), e.g. an
    MNA pivot order (ggmres.matrices.mna_pivot_order)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    rng = np.random.default_rng(seed)
    prow = rng.permutation(n).astype(np.int32)
    if identity_perm:
        prow = np.arange(n, dtype=np.int32)
    pcol = np.argsort(prow).astype(np.int32)
    if perm is not None:
        prow, pcol = (np.asarray(p, np.int32) for p in perm)
    lscale = rng.uniform(0.5, 2.0, n)
    rscale = rng.uniform(0.5, 2.0, n)
    middle = rng.uniform(0.5, 2.0, n)
    d1 = rng.uniform(0.5, 2.0, n)
    Pr = sp.csr_matrix((np.ones(n), (np.arange(n), prow)), shape=(n, n))
    Pc = sp.csr_matrix((np.ones(n), (np.arange(n), pcol)), shape=(n, n))
    B = (Pr @ sp.diags(1.0 / lscale) @ A @ sp.diags(1.0 / rscale) @ Pc).tocsr()
    B.sort_indices()
    Lt, Ut = O.ilu0(B)
    Ls = csr_sp(Lt) @ sp.diags(d1)
    Us = sp.diags(middle / d1) @ csr_sp(Ut)
    L = O.csr(Ls)
    U = O.csr(Us)
    return O.Split(L, U, middle, prow, pcol, lscale, rscale)


def netlist_system(path, grid, pad_stride):
    """The bench's netlist workload at test size (bench.py netlist_system): a
    synthetic IBM-PG-style netlist (ggmres.matrices.pg_netlist) through the
    library's SPICE front end into MNA, A = G + C/h; returns (A, prow, pcol,
    tail rows = 2 * pads) with the MNA pivot order (pads and branch rows first)."""
    from ggmres import host as H, matrices as M
    ng, npad = M.pg_netlist(path, grid, grid, pad_stride=pad_stride)
    nl = H.Netlist(path)
    A = (nl.G + nl.C / nl.tstep).tocsr()
    A.sort_indices()
    prow, pcol = M.mna_pivot_order(ng, npad, A.shape[0])
    return A, prow, pcol, 2 * npad


def rel_err(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    d = np.linalg.norm(a - b)
    s = np.linalg.norm(b)
    return d / s if s else d


def hist_close(h_test, h_ref, rtol):
    """Residual histories equal in length and within rtol elementwise (relative)."""
    h_test = np.asarray(h_test)
    h_ref = np.asarray(h_ref)
    if h_test.shape != h_ref.shape:
        return False, f"length {h_test.shape} vs {h_ref.shape}"
    denom = np.maximum(np.abs(h_ref), 1e-300)
    dev = np.max(np.abs(h_test - h_ref) / denom) if h_ref.size else 0.0
    return dev <= rtol, f"max rel dev {dev:.3e}"


# ---- the device vector space (DESIGN.md "Wavefront layout", "Reduction order")
def device_layout(n, nx=None, ny=None, skew=1, border=0):
    """(lay2nat, G) of the solver's vector space: natural order, or -- for a 2D
    grid of line length nx on the wavefront path -- band = j//64, lane l = j%64,
    step t = i + skew*l + skew-1, slot ((band*T/2 + t//2)*64 + l)*2 + t%2 with
    T = roundup(nx + 63*skew + 2*(skew-1), 32) (skew = k+1 for ILU(k) factors
    of a 5-point grid); for a 3D grid (ny given) 8-line x 8-plane tiles; padded to a multiple of 512 slots; G = min(1024, ceil(Ppad/2 / 1024)), or 512 beyond 2M units
    reduction blocks.  border: a bordered grid (gg_internal.h Wave2D::bnt) --
    rows [0, border) at slots [0, border), the grid rows after them at
    roundup(border, 64) + their 2D slot."""
    n_all, n = n, n - border
    if nx is None:
        P = n
        slots = np.arange(n, dtype=np.int64)
    elif ny is not None and n // (nx * ny) >= 2:
        # 3D: 8-line x 8-plane tiles (gg_internal.h Wave2D::slot, tile = true):
        # lane a + 8*g(c), g(c) = c ^ (c >> 1); step t = i + a + c;
        # T = roundup(nx + 14, 16); tiles K-major
        nxy = nx * ny
        nz = n // nxy
        NJ, NK = (ny + 7) // 8, (nz + 7) // 8
        T = (nx + 14 + 15) // 16 * 16
        P = NJ * NK * T * 64
        r = np.arange(n, dtype=np.int64)
        k, q = r // nxy, r % nxy
        j, i = q // nx, q % nx
        a, c = j % 8, k % 8
        lane = a + 8 * (c ^ (c >> 1))
        t = i + a + c
        band = (k // 8) * NJ + j // 8
        slots = ((band * (T // 2) + t // 2) * 64 + lane) * 2 + t % 2
    else:
        nxy = n if ny is None else nx * ny
        ny = nxy // nx
        nz = n // nxy
        T = (nx + 63 * skew + 2 * (skew - 1) + 31) // 32 * 32
        nb = (ny + 63) // 64
        P2 = nb * T * 64
        P = nz * P2
        r = np.arange(n, dtype=np.int64)
        k, q = r // nxy, r % nxy
        j, i = q // nx, q % nx
        lane = j % 64
        t = i + skew * lane + (skew - 1)
        slots = k * P2 + (((j // 64) * (T // 2) + t // 2) * 64 + lane) * 2 + t % 2
    if border:
        bofs = (border + 63) // 64 * 64
        slots = np.concatenate([np.arange(border, dtype=np.int64), bofs + slots])
        P += bofs
    n = n_all
    ppad = max((max(P, 1) + 511) // 512 * 512, 512)
    lay2nat = np.full(ppad, -1, np.int64)
    lay2nat[slots] = np.arange(n, dtype=np.int64)
    units = ppad // 2
    # kernels.hip reduce_grid: beyond 8 units per thread at 1024 blocks, kWideG = 512
    G = 512 if units > 1024 * 256 * 8 else min(1024, max(1, (units + 1023) // 1024))
    return lay2nat, G
