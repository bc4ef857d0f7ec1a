"""ctypes binding of the fp64 oracle (oracle.c).

TEST INFRASTRUCTURE ONLY.  Importable from tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never from the product package.
"""
import ctypes
import os
import subprocess
from collections import namedtuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_LIB_MT = os.path.join(_HERE, "liboracle_mt.so")   # bench.py cpu_baseline_mt only (OpenMP loops)
_lib = None
_libs = {}

CSR = namedtuple("CSR", "n rp ci v")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_PI = ctypes.POINTER(ctypes.c_int)
_PD = ctypes.POINTER(ctypes.c_double)


class SplitT(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int),
        ("l_rp", _PI), ("l_ci", _PI), ("l_v", _PD),
        ("u_rp", _PI), ("u_ci", _PI), ("u_v", _PD),
        ("middle", _PD), ("lscale", _PD), ("rscale", _PD),
        ("perm_row", _PI), ("perm_col", _PI),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def use_mt(on):
    """Route the oracle calls to liboracle_mt.so (OpenMP SpMV / BLAS-1 / update
    loops, serial triangular solves; another reduction order -- a timing
    baseline, never a checker) or back to the serial checker."""
    global _lib
    _lib = None
    _load(_LIB_MT if on else _LIB)


def threads():
    """threads the loaded oracle library runs its loops on (1 = the serial checker)"""
    return int(lib().orc_threads())


def lib():
    if _lib is None:
        _load(_LIB)
    return _lib


def _load(path):
    global _lib
    if path in _libs:
        _lib = _libs[path]
        return
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(
            os.path.join(_HERE, "oracle.c")):
        build()
    L = ctypes.CDLL(path)
    L.orc_spmv.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _f64p, _f64p]
    L.orc_residual.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _f64p, _f64p, _f64p]
    for f in (L.orc_ilu0,):
        f.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p,
                      _i32p, ctypes.POINTER(_PI), ctypes.POINTER(_PD),
                      _i32p, ctypes.POINTER(_PI), ctypes.POINTER(_PD)]
        f.restype = ctypes.c_int
    L.orc_ilu0_values.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _f64p]
    L.orc_iluk.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p,
                           _i32p, ctypes.POINTER(_PI), ctypes.POINTER(_PD),
                           _i32p, ctypes.POINTER(_PI), ctypes.POINTER(_PD)]
    L.orc_iluk.restype = ctypes.c_int
    L.orc_free.argtypes = [ctypes.c_void_p]
    L.orc_lusolve.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _i32p, _i32p, _f64p,
                              _f64p, _f64p]
    for f in (L.orc_split_left, L.orc_split_right, L.orc_split_start):
        f.argtypes = [ctypes.POINTER(SplitT), _f64p, _f64p]
    L.orc_set_dot_order.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                    ctypes.c_void_p]
    L.orc_set_dot_order_shards.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p]
    L.orc_canon_trsv.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p, _f64p,
                                 _f64p, _f64p]
    L.orc_sub_seq.argtypes = [ctypes.c_int, _i32p, _i32p, _f64p, _f64p, _f64p, _f64p]
    L.orc_gen_rot.argtypes = [ctypes.c_double, ctypes.c_double, _PD, _PD]
    L.orc_set_div_mode.argtypes = [ctypes.c_int, ctypes.c_int]
    L.orc_set_fma_tail.argtypes = [ctypes.c_int]
    L.orc_set_orth.argtypes = [ctypes.c_int]
    L.orc_apply_rot.argtypes = [_PD, _PD, ctypes.c_double, ctypes.c_double]
    common = [_f64p, _f64p, ctypes.c_int, _PI, _PD, _f64p, ctypes.c_int, _PI, _PI]
    L.orc_gmres_left.argtypes = ([ctypes.c_int, _i32p, _i32p, _f64p,
                                  _i32p, _i32p, _f64p, _i32p, _i32p, _f64p] + common)
    L.orc_gmres_left.restype = ctypes.c_int
    L.orc_gmres_split.argtypes = ([ctypes.c_int, _i32p, _i32p, _f64p,
                                   ctypes.POINTER(SplitT)] + common)
    L.orc_gmres_split.restype = ctypes.c_int
    _libs[path] = L
    _lib = L


def csr(A):
    """scipy.sparse matrix (or CSR tuple) -> oracle CSR with sorted int32 indices."""
    if isinstance(A, CSR):
        return A
    A = A.tocsr()
    A.sort_indices()
    return CSR(A.shape[0], np.ascontiguousarray(A.indptr, dtype=np.int32),
               np.ascontiguousarray(A.indices, dtype=np.int32),
               np.ascontiguousarray(A.data, dtype=np.float64))


def spmv(A, x):
    A = csr(A)
    y = np.zeros(A.n)
    lib().orc_spmv(A.n, A.rp, A.ci, A.v, np.ascontiguousarray(x, np.float64), y)
    return y


def residual(A, x, b):
    A = csr(A)
    r = np.zeros(A.n)
    lib().orc_residual(A.n, A.rp, A.ci, A.v, np.ascontiguousarray(x, np.float64),
                       np.ascontiguousarray(b, np.float64), r)
    return r


def _take(n, rp, ci_p, v_p):
    nnz = int(rp[n])
    ci = np.ctypeslib.as_array(ci_p, shape=(max(nnz, 1),))[:nnz].copy()
    v = np.ctypeslib.as_array(v_p, shape=(max(nnz, 1),))[:nnz].copy()
    lib().orc_free(ctypes.cast(ci_p, ctypes.c_void_p))
    lib().orc_free(ctypes.cast(v_p, ctypes.c_void_p))
    return CSR(n, rp, ci.astype(np.int32), v)


def ilu0(A):
    """leftILU restated (src/leftILU.cu:27-336) -> (L, U)."""
    A = csr(A)
    n = A.n
    l_rp = np.zeros(n + 1, np.int32)
    u_rp = np.zeros(n + 1, np.int32)
    lci, lv, uci, uv = _PI(), _PD(), _PI(), _PD()
    rc = lib().orc_ilu0(n, A.rp, A.ci, A.v, l_rp, ctypes.byref(lci), ctypes.byref(lv),
                        u_rp, ctypes.byref(uci), ctypes.byref(uv))
    assert rc == 0
    return _take(n, l_rp, lci, lv), _take(n, u_rp, uci, uv)


def ilu0_values(A):
    """leftILU's factored matrix before the split (A's sorted CSR order)."""
    A = csr(A)
    out = np.zeros(max(int(A.rp[A.n]), 1))
    assert lib().orc_ilu0_values(A.n, A.rp, A.ci, A.v, out) == 0
    return out[:int(A.rp[A.n])]


def iluk(A, k):
    """ITSOL lofC+ilukC restated (src/iluk.cpp:56-334) -> (L, U); raises on zero pivot."""
    A = csr(A)
    n = A.n
    l_rp = np.zeros(n + 1, np.int32)
    u_rp = np.zeros(n + 1, np.int32)
    lci, lv, uci, uv = _PI(), _PD(), _PI(), _PD()
    rc = lib().orc_iluk(int(k), n, A.rp, A.ci, A.v, l_rp, ctypes.byref(lci), ctypes.byref(lv),
                        u_rp, ctypes.byref(uci), ctypes.byref(uv))
    if rc != 0:
        raise ZeroDivisionError("ILU(k): zero pivot (iluk.cpp:175-185)")
    return _take(n, l_rp, lci, lv), _take(n, u_rp, uci, uv)


def lusolve(L, U, y):
    x = np.zeros(L.n)
    lib().orc_lusolve(L.n, L.rp, L.ci, L.v, U.rp, U.ci, U.v,
                      np.ascontiguousarray(y, np.float64), x)
    return x


class Split:
    """ILU++-style split preconditioner arrays (PG boundary)."""

    def __init__(self, L, U, middle, perm_row, perm_col, lscale, rscale):
        self.L, self.U = L, U
        self.middle = np.ascontiguousarray(middle, np.float64)
        self.lscale = np.ascontiguousarray(lscale, np.float64)
        self.rscale = np.ascontiguousarray(rscale, np.float64)
        self.perm_row = np.ascontiguousarray(perm_row, np.int32)
        self.perm_col = np.ascontiguousarray(perm_col, np.int32)
        c = lambda a, t: a.ctypes.data_as(t)
        self.s = SplitT(L.n, c(L.rp, _PI), c(L.ci, _PI), c(L.v, _PD),
                        c(U.rp, _PI), c(U.ci, _PI), c(U.v, _PD),
                        c(self.middle, _PD), c(self.lscale, _PD), c(self.rscale, _PD),
                        c(self.perm_row, _PI), c(self.perm_col, _PI))

    def _apply(self, f, v):
        out = np.zeros(self.L.n)
        f(ctypes.byref(self.s), np.ascontiguousarray(v, np.float64), out)
        return out

    def left(self, v):
        return self._apply(lib().orc_split_left, v)

    def right(self, v):
        return self._apply(lib().orc_split_right, v)

    def start(self, v):
        return self._apply(lib().orc_split_start, v)


_dot_keep = None


def set_dot_order(lay2nat=None, G=1):
    """None: serial dots (reference CPU engine).  Otherwise restate the device
    reduction tree over the slot->natural map lay2nat (int64, -1 = padding)."""
    global _dot_keep
    if lay2nat is None:
        _dot_keep = None
        lib().orc_set_dot_order(0, 0, 1, None)
    else:
        _dot_keep = np.ascontiguousarray(lay2nat, np.int64)
        lib().orc_set_dot_order(1, len(_dot_keep), int(G), _dot_keep.ctypes.data)


def set_dot_order_shards(segments, G):
    """The sharded solve's tree (gpu-gmres_amd/csrc/dd.hip): segments = per
    shard, its dot range's slot -> index map (int64, -1 = padding); each shard
    sums its range into G block partials, then all shards' partials are summed
    shard-major as in the single-device tree."""
    global _dot_keep
    seglen = np.array([len(s) for s in segments], np.int64)
    cat = np.ascontiguousarray(np.concatenate(segments), np.int64)
    _dot_keep = (seglen, cat)
    lib().orc_set_dot_order_shards(len(segments), seglen.ctypes.data, int(G), cat.ctypes.data)


def set_div_mode(mul_l=False, mul_u=False):
    """Division of the non-unit triangles: False / 0 = x / d (the reference),
    True / 1 = x * (1.0 / d) (the device's GG_DIV_RCP on a wavefront triangle),
    2 = the device's GG_DIV_FMA rows (lusolve only: b and the coefficients
    pre-scaled by 1.0 / d, the nearest term first, fused multiply-adds); for
    order-matched checks only -- reset with set_div_mode()."""
    lib().orc_set_div_mode(int(mul_l), int(mul_u))


def set_fma_tail(tail=0):
    """GG_DIV_FMA on a bordered grid (split engine): the Ml rows below the
    first `tail` rows take their tail-column terms first (canonical order),
    then the rest nearest first -- as the device forms them (k_border_sub
    before the mesh wavefront).  0 (default) = every row nearest first."""
    lib().orc_set_fma_tail(int(tail))


def set_orth(cgs2=False):
    """False: modified Gram-Schmidt (the reference); True: CGS2, the sharded
    solve's GG_SOLVE_CGS2 restated (reset with set_orth())."""
    lib().orc_set_orth(int(bool(cgs2)))


def gen_rot(dx, dy):
    cs, sn = ctypes.c_double(), ctypes.c_double()
    lib().orc_gen_rot(dx, dy, ctypes.byref(cs), ctypes.byref(sn))
    return cs.value, sn.value


def _gmres_out(ret, x, mi, tl, hist, hl, inner):
    return dict(ret=ret, x=x, iters=mi.value, relres=tl.value,
                hist=hist[:hl.value].copy(), inner=inner.value)


def gmres_left(A, L, U, b, x0=None, m=30, max_iter=3000, tol=1e-10, hist_cap=None):
    """GMRES_leftILU0 restated (src/gmres.cu:566-717)."""
    A = csr(A)
    x = np.zeros(A.n) if x0 is None else np.array(x0, np.float64, copy=True)
    cap = hist_cap or (max_iter + max_iter // max(m, 1) + 8)
    hist = np.zeros(cap)
    mi, tl, hl, inner = ctypes.c_int(max_iter), ctypes.c_double(tol), ctypes.c_int(), ctypes.c_int()
    ret = lib().orc_gmres_left(A.n, A.rp, A.ci, A.v, L.rp, L.ci, L.v, U.rp, U.ci, U.v,
                               np.ascontiguousarray(b, np.float64), x, int(m),
                               ctypes.byref(mi), ctypes.byref(tl), hist, cap,
                               ctypes.byref(hl), ctypes.byref(inner))
    return _gmres_out(ret, x, mi, tl, hist, hl, inner)


def gmres_split(A, P, b, x0=None, m=32, max_iter=10000, tol=1e-7, hist_cap=None):
    """GMRESilu restated (src/gmres.cu:2069-2252) with a Split preconditioner."""
    A = csr(A)
    x = np.zeros(A.n) if x0 is None else np.array(x0, np.float64, copy=True)
    cap = hist_cap or (max_iter + max_iter // max(m, 1) + 8)
    hist = np.zeros(cap)
    mi, tl, hl, inner = ctypes.c_int(max_iter), ctypes.c_double(tol), ctypes.c_int(), ctypes.c_int()
    ret = lib().orc_gmres_split(A.n, A.rp, A.ci, A.v, ctypes.byref(P.s),
                                np.ascontiguousarray(b, np.float64), x, int(m),
                                ctypes.byref(mi), ctypes.byref(tl), hist, cap,
                                ctypes.byref(hl), ctypes.byref(inner))
    return _gmres_out(ret, x, mi, tl, hist, hl, inner)


# ---------------------------------------------------------------- transient (C5)
def pulse(q, it, h):
    """PULSE source value at time index it (gen_PULSEut_kernel, src/kernels.cu:223-245)."""
    f = lib().orc_pulse
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_double]
    q = np.ascontiguousarray(q, np.float64)
    return f(q.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(it), float(h))


def pwl(tv, it, h):
    """PWL source value at time index it (gen_PWLut_kernel, src/kernels.cu:146-176);
    tv = [t0, v0, t1, v1, ...]; holds v0 before t0 (the reference reads v[-1])."""
    f = lib().orc_pwl
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_double]
    tv = np.ascontiguousarray(tv, np.float64)
    return f(tv.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), len(tv) // 2, int(it), float(h))


SRC_DC, SRC_PULSE, SRC_PWL = 0, 1, 2   # include/ggmres.h gg_src_kind


def source_value(kind, data, it, h):
    """One source at time index it: DC (gen_dcVt_kernel, src/kernels.cu:73-85: the
    constant), PULSE (gen_PULSEut_kernel) or PWL (gen_PWLut_kernel)."""
    if kind == SRC_DC:
        return float(data[0])
    if kind == SRC_PULSE:
        return pulse(data, it, h)
    if kind == SRC_PWL:
        return pwl(data, it, h)
    raise ValueError(kind)


def transient_rhs(cdiag, src_node, u, x):
    """w = B u + (C/h) x as the reference step driver forms it."""
    n = len(x)
    w = np.zeros(n)
    src_node = np.ascontiguousarray(src_node, np.int32)
    f = lib().orc_transient_rhs
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    u = np.ascontiguousarray(u, np.float64)
    c = np.ascontiguousarray(cdiag, np.float64)
    xx = np.ascontiguousarray(x, np.float64)
    f(n, len(src_node), src_node.ctypes.data, u.ctypes.data, c.ctypes.data, xx.ctypes.data,
      w.ctypes.data)
    return w


def transient(A, L, U, nsteps, h, cdiag, src_node, pulses, ports, x0, m=32, max_iter=10000,
              tol=1e-7, sources=None, taps=None):
    """The reference's backward-Euler step driver (src/mna_solve_gpu_gmres.cpp:564-647)
    with GMRES_leftILU0 per step, warm start x_{t-1}; returns dict(x, ports, iters_total).
    Sources: PULSE parameter rows `pulses`, or `sources` = [(kind, data), ...]."""
    x = np.array(x0, np.float64, copy=True)
    if sources is None:
        sources = [(SRC_PULSE, q) for q in np.asarray(pulses, np.float64).reshape(-1, 7)]
    ports = np.asarray(ports, np.int64)
    pv = np.zeros((len(ports), nsteps + 1))
    pv[:, 0] = x[ports]
    total = 0
    ret = 0
    if taps is not None:     # ir_info (src/mna_solve_gpu_gmres.cpp:285-292, 633-645, 780-797)
        taps = np.asarray(taps, np.int64)
        tmax, tmin, tsum = x[taps].copy(), x[taps].copy(), x[taps].copy()
    for it in range(1, nsteps + 1):
        u = np.array([source_value(k, q, it, h) for k, q in sources])
        w = transient_rhs(cdiag, src_node, u, x)
        o = gmres_left(A, L, U, w, x0=x, m=m, max_iter=max_iter, tol=tol)
        x = o["x"]
        total += o["iters"]
        ret = ret or o["ret"]
        pv[:, it] = x[ports]
        if taps is not None:
            for j, t in enumerate(taps):
                v = x[t]
                if tmax[j] < v:
                    tmax[j] = v
                if v < tmin[j]:
                    tmin[j] = v
                tsum[j] += v
    out = dict(x=x, ports=pv, iters_total=total, ret=ret)
    if taps is not None:
        out["taps"] = (tmax, tmin, tsum / (nsteps + 1), tmax - tmin)
    return out


def gaxpy_csc(A, x, y):
    """cs_dl_gaxpy restated: y += A x, A (scipy) in compressed columns, column by column."""
    import scipy.sparse as sp
    A = sp.csc_matrix(A)
    p = np.ascontiguousarray(A.indptr, np.int64)
    i = np.ascontiguousarray(A.indices, np.int64)
    v = np.ascontiguousarray(A.data, np.float64)
    f = lib().orc_gaxpy_csc
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    xx = np.ascontiguousarray(x, np.float64)
    assert y.dtype == np.float64 and y.flags.c_contiguous
    f(A.shape[1], p.ctypes.data, i.ctypes.data, v.ctypes.data, xx.ctypes.data, y.ctypes.data)
    return y


def transient_mna(A, L, U, it0, nsteps, h, R, B, sources, ports, x0, m=32, max_iter=10000, tol=1e-7):
    """The step driver with a general MNA right-hand side (src/mna_solve_gpu_gmres.cpp:585-591:
    w = 0; cs_dl_gaxpy(B, u, w); xnr = 0; cs_dl_gaxpy(right, xn, xnr); w += xnr), sources at
    time index it0 + j - 1 for step j; R None = 0 (a DC point).  GMRES_leftILU0 per step,
    warm start.  Returns dict(x, ports [nport, nsteps+1], iters_total, ret)."""
    x = np.array(x0, np.float64, copy=True)
    n = len(x)
    ports = np.asarray(ports, np.int64)
    pv = np.zeros((len(ports), nsteps + 1))
    pv[:, 0] = x[ports]
    total, ret = 0, 0
    for j in range(1, nsteps + 1):
        it = it0 + j - 1
        u = np.array([source_value(k, q, it, h) for k, q in sources])
        w = gaxpy_csc(B, u, np.zeros(n))
        xnr = np.zeros(n)
        if R is not None:
            gaxpy_csc(R, x, xnr)
        w += xnr
        o = gmres_left(A, L, U, w, x0=x, m=m, max_iter=max_iter, tol=tol)
        x = o["x"]
        total += o["iters"]
        ret = ret or o["ret"]
        pv[:, j] = x[ports]
    return dict(x=x, ports=pv, iters_total=total, ret=ret)
