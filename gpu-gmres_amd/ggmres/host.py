"""Host-only entry points of libggmres.so (include/ggmres_host.h): domain
decomposition setup and Matrix Market input.  No GPU is needed."""
import ctypes

import numpy as np
import scipy.sparse as sp

from . import _check, _csr_arrays, lib

PART_BISECT, PART_BLOCKS, PART_GRID, PART_COLOR_SEP = 0, 1, 2, 4
_PI = ctypes.POINTER(ctypes.c_int)
_PD = ctypes.POINTER(ctypes.c_double)


def _ptr(a, t):
    return a.ctypes.data_as(t)


def _take_csr(nrows, ncols, rp, ci_p, v_p):
    L = lib()
    nnz = int(rp[nrows])
    ci = np.ctypeslib.as_array(ci_p, (max(nnz, 1),))[:nnz].copy()
    v = np.ctypeslib.as_array(v_p, (max(nnz, 1),))[:nnz].copy()
    L.gg_host_free(ctypes.cast(ci_p, ctypes.c_void_p))
    L.gg_host_free(ctypes.cast(v_p, ctypes.c_void_p))
    return sp.csr_matrix((v, ci, np.asarray(rp, np.int32)), shape=(nrows, ncols))


def partition(A, nparts, method=PART_BISECT):
    """partition4 (src/partition3.cpp:122-194) -> dict(node_part, part_size,
    pinv, q, begin): nparts interiors, separator part nparts last."""
    n, rp, ci, _ = _csr_arrays(A)
    node_part = np.zeros(n, np.int32)
    part_size = np.zeros(nparts + 1, np.int32)
    pinv = np.zeros(n, np.int32)
    q = np.zeros(n, np.int32)
    _check(lib().gg_host_partition(ctypes.c_int(n), _ptr(rp, _PI), _ptr(ci, _PI), ctypes.c_int(nparts),
                                   ctypes.c_int(method), _ptr(node_part, _PI), _ptr(part_size, _PI),
                                   _ptr(pinv, _PI), _ptr(q, _PI)))
    begin = np.concatenate([[0], np.cumsum(part_size)]).astype(np.int64)
    return dict(node_part=node_part, part_size=part_size, pinv=pinv, q=q, begin=begin)


def permute(A, pinv, q):
    """P A P^T for (pinv, q) of partition()."""
    n, rp, ci, v = _csr_arrays(A)
    pinv = np.ascontiguousarray(pinv, np.int32)
    q = np.ascontiguousarray(q, np.int32)
    brp = np.zeros(n + 1, np.int32)
    bci, bv = _PI(), _PD()
    _check(lib().gg_host_permute(ctypes.c_int(n), _ptr(rp, _PI), _ptr(ci, _PI), _ptr(v, _PD),
                                 _ptr(pinv, _PI), _ptr(q, _PI), _ptr(brp, _PI), ctypes.byref(bci),
                                 ctypes.byref(bv)))
    return _take_csr(n, n, brp, bci, bv)


def block(A, r0, r1, c0, c1):
    """rows [r0, r1) x cols [c0, c1) (dd_form's As / E / F / At, src/form_dd.cpp:32-110)."""
    n, rp, ci, v = _csr_arrays(A)
    brp = np.zeros(r1 - r0 + 1, np.int32)
    bci, bv = _PI(), _PD()
    _check(lib().gg_host_block(ctypes.c_int(n), _ptr(rp, _PI), _ptr(ci, _PI), _ptr(v, _PD),
                               ctypes.c_int(r0), ctypes.c_int(r1), ctypes.c_int(c0), ctypes.c_int(c1),
                               _ptr(brp, _PI), ctypes.byref(bci), ctypes.byref(bv)))
    return _take_csr(r1 - r0, c1 - c0, brp, bci, bv)


def dd_form(B, begin, nparts):
    """dd_form's blocks of the permuted matrix B: As[k], E[k] (interior k x
    separator), F[k] (separator x interior k), At (separator x separator)."""
    s0, s1 = int(begin[nparts]), int(begin[nparts + 1])
    As = [block(B, int(begin[k]), int(begin[k + 1]), int(begin[k]), int(begin[k + 1])) for k in range(nparts)]
    E = [block(B, int(begin[k]), int(begin[k + 1]), s0, s1) for k in range(nparts)]
    F = [block(B, s0, s1, int(begin[k]), int(begin[k + 1])) for k in range(nparts)]
    return As, E, F, block(B, s0, s1, s0, s1)


def read_mtx(path, expand_symmetric=False):
    """Matrix Market -> scipy CSR (readSparseMatrix, src_thermal/SpMV_gen.cpp:93-187)."""
    nr, nc = ctypes.c_int(), ctypes.c_int()
    rp_p, ci_p, v_p = _PI(), _PI(), _PD()
    _check(lib().gg_host_read_mtx(str(path).encode(), ctypes.c_int(int(expand_symmetric)),
                                  ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(rp_p),
                                  ctypes.byref(ci_p), ctypes.byref(v_p)))
    rp = np.ctypeslib.as_array(rp_p, (nr.value + 1,)).copy()
    lib().gg_host_free(ctypes.cast(rp_p, ctypes.c_void_p))
    return _take_csr(nr.value, nc.value, rp, ci_p, v_p)


# ---- sharded-solve plan (gg_host_dd_*): the pieces each shard of
# include/ggmres_dd.h runs on, in the shard's local index space
# [interior (nI) | separator (nS) | halo (nparts * max_iface)]
DD_A, DD_LI, DD_LS, DD_LSH, DD_UI, DD_US, DD_UIS = range(7)


class DDPlan:
    def __init__(self, A, nparts, method=PART_BLOCKS):
        n, rp, ci, v = _csr_arrays(A)
        h = ctypes.c_void_p()
        L = lib()
        L.gg_host_dd_plan.argtypes = [ctypes.c_int, _PI, _PI, _PD, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p)]
        for f in ("gg_host_dd_plan_sizes", "gg_host_dd_plan_perm", "gg_host_dd_shard_sizes",
                  "gg_host_dd_shard_csr", "gg_host_dd_shard_div", "gg_host_dd_shard_index",
                  "gg_host_dd_plan_free"):
            getattr(L, f).restype = ctypes.c_int if f != "gg_host_dd_plan_free" else None
        _check(L.gg_host_dd_plan(ctypes.c_int(n), _ptr(rp, _PI), _ptr(ci, _PI), _ptr(v, _PD),
                                 ctypes.c_int(nparts), ctypes.c_int(method), ctypes.byref(h)))
        self.h = h
        s = np.zeros(4, np.int32)
        _check(L.gg_host_dd_plan_sizes(h, _ptr(s, _PI)))
        self.n, self.P, self.nsep, self.max_iface = (int(x) for x in s)
        self.part_size = np.zeros(self.P + 1, np.int32)
        self.pinv = np.zeros(self.n, np.int32)
        self.q = np.zeros(self.n, np.int32)
        _check(L.gg_host_dd_plan_perm(h, _ptr(self.part_size, _PI), _ptr(self.pinv, _PI),
                                      _ptr(self.q, _PI)))
        self.begin = np.concatenate([[0], np.cumsum(self.part_size)]).astype(np.int64)

    def close(self):
        if self.h:
            lib().gg_host_dd_plan_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def shard(self, p):
        """dict: nI, nS, A, LI, LS, LSH, UI, US, UIS (scipy CSR, entries in the
        reference's summation order), dLI/dLS/dUI/dUS (divisors), iface, rows."""
        L = lib()
        sz = np.zeros(3, np.int32)
        _check(L.gg_host_dd_shard_sizes(self.h, ctypes.c_int(p), _ptr(sz, _PI)))
        nI, nS, ni = (int(x) for x in sz)
        ncols = {DD_A: nI + nS + self.P * self.max_iface, DD_LI: nI, DD_LS: nS,
                 DD_LSH: self.P * self.max_iface, DD_UI: nI, DD_US: nS, DD_UIS: nS}
        out = dict(nI=nI, nS=nS)
        for name, piece in (("A", DD_A), ("LI", DD_LI), ("LS", DD_LS), ("LSH", DD_LSH),
                            ("UI", DD_UI), ("US", DD_US), ("UIS", DD_UIS)):
            nr = ctypes.c_int()
            rp_p, ci_p, v_p = _PI(), _PI(), _PD()
            _check(L.gg_host_dd_shard_csr(self.h, ctypes.c_int(p), ctypes.c_int(piece),
                                          ctypes.byref(nr), ctypes.byref(rp_p), ctypes.byref(ci_p),
                                          ctypes.byref(v_p)))
            rp = np.ctypeslib.as_array(rp_p, (nr.value + 1,)).copy()
            L.gg_host_free(ctypes.cast(rp_p, ctypes.c_void_p))
            out[name] = _take_csr(nr.value, max(ncols[piece], 1), rp, ci_p, v_p)
        for name, piece, nr in (("dLI", DD_LI, nI), ("dLS", DD_LS, nS), ("dUI", DD_UI, nI),
                                ("dUS", DD_US, nS)):
            d = np.zeros(max(nr, 1))
            _check(L.gg_host_dd_shard_div(self.h, ctypes.c_int(p), ctypes.c_int(piece), _ptr(d, _PD)))
            out[name] = d[:nr]
        iface = np.zeros(max(ni, 1), np.int32)
        rows = np.zeros(max(nI + nS, 1), np.int32)
        _check(L.gg_host_dd_shard_index(self.h, ctypes.c_int(p), _ptr(iface, _PI), _ptr(rows, _PI)))
        out["iface"] = iface[:ni]
        out["rows"] = rows[:nI + nS]
        return out


# ---- SPICE power-grid netlist -> MNA (gg_host_read_netlist)
class _Netlist(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int), ("n_l", ctypes.c_int), ("n_v", ctypes.c_int),
                ("n_i", ctypes.c_int), ("n", ctypes.c_int), ("tstep", ctypes.c_double),
                ("tstop", ctypes.c_double),
                ("g_row_ptr", _PI), ("g_col_idx", _PI), ("g_val", _PD),
                ("c_row_ptr", _PI), ("c_col_idx", _PI), ("c_val", _PD),
                ("b_row_ptr", _PI), ("b_col_idx", _PI), ("b_val", _PD),
                ("src_kind", _PI), ("src_ptr", _PI), ("src_data", _PD),
                ("nport", ctypes.c_int), ("port", _PI)]


class Netlist:
    """The MNA system of a flat SPICE power-grid netlist (parser() + stampG /
    stampC / stampB, src/parser.cpp:69-272, 1904-2886): G, C (n x n) and B
    (n x nsrc) as scipy CSR, sources [(kind, params)] (V first, then I),
    tstep, tstop, ports (unknown indices, -1 = ground / unknown)."""

    def __init__(self, path):
        nl = _Netlist()
        L = lib()
        L.gg_host_read_netlist.argtypes = [ctypes.c_char_p, ctypes.POINTER(_Netlist)]
        L.gg_host_free_netlist.argtypes = [ctypes.POINTER(_Netlist)]
        L.gg_host_free_netlist.restype = None
        _check(L.gg_host_read_netlist(str(path).encode(), ctypes.byref(nl)))
        try:
            n = nl.n
            self.n, self.n_nodes, self.n_l, self.n_v, self.n_i = n, nl.n_nodes, nl.n_l, nl.n_v, nl.n_i
            self.tstep, self.tstop = nl.tstep, nl.tstop
            nsrc = nl.n_v + nl.n_i

            def csr(rp_p, ci_p, v_p, ncols):
                rp = np.ctypeslib.as_array(rp_p, (n + 1,)).copy()
                nnz = int(rp[-1])
                ci = np.ctypeslib.as_array(ci_p, (max(nnz, 1),))[:nnz].copy()
                v = np.ctypeslib.as_array(v_p, (max(nnz, 1),))[:nnz].copy()
                return sp.csr_matrix((v, ci, rp), shape=(n, ncols))

            self.G = csr(nl.g_row_ptr, nl.g_col_idx, nl.g_val, n)
            self.C = csr(nl.c_row_ptr, nl.c_col_idx, nl.c_val, n)
            self.B = csr(nl.b_row_ptr, nl.b_col_idx, nl.b_val, nsrc)
            kind = np.ctypeslib.as_array(nl.src_kind, (max(nsrc, 1),))[:nsrc].copy()
            ptr = np.ctypeslib.as_array(nl.src_ptr, (nsrc + 1,)).copy()
            data = np.ctypeslib.as_array(nl.src_data, (max(int(ptr[-1]), 1),))[:int(ptr[-1])].copy()
            self.sources = [(int(kind[k]), data[ptr[k]:ptr[k + 1]].copy()) for k in range(nsrc)]
            self.ports = np.ctypeslib.as_array(nl.port, (max(nl.nport, 1),))[:nl.nport].copy()
        finally:
            L.gg_host_free_netlist(ctypes.byref(nl))

    def transient_inputs(self, h):
        """(A = G + C/h, cdiag = diag(C)/h, src_node, src_kind, src_ptr, src_data)
        for Solver.transient_src.  Needs a diagonal C and one +-1 entry per
        source column of B; a -1 entry negates the source's values (exact)."""
        from . import SRC_DC, SRC_PULSE
        C = self.C.tocoo()
        if np.any(C.row != C.col):
            raise ValueError("C is not diagonal (capacitors between two non-ground nodes)")
        Bc = self.B.tocsc()
        cdiag = np.zeros(self.n)
        cdiag[C.row] = C.data / h
        nodes, kinds, ptr, data = [], [], [0], []
        for k, (kind, par) in enumerate(self.sources):
            lo, hi = Bc.indptr[k], Bc.indptr[k + 1]
            if hi - lo != 1 or abs(Bc.data[lo]) != 1.0:
                raise ValueError(f"source {k}: B column is not a single +-1 entry")
            sgn = Bc.data[lo]
            par = np.array(par, dtype=np.float64)
            if sgn < 0:
                if kind == SRC_DC:
                    par = -par
                elif kind == SRC_PULSE:
                    par[:2] = -par[:2]
                else:
                    par[1::2] = -par[1::2]
            nodes.append(int(Bc.indices[lo]))
            kinds.append(kind)
            data.extend(par.tolist())
            ptr.append(len(data))
        A = (self.G + sp.diags(cdiag)).tocsr()
        A.sort_indices()
        return (A, cdiag, np.array(nodes, np.int32), np.array(kinds, np.int32),
                np.array(ptr, np.int32), np.array(data, np.float64))
