"""ggmres -- Python binding of libggmres.so (the MI355X GMRES solver C ABI).

Thin ctypes layer over include/ggmres.h: every call goes through the C ABI
into the hand-written HIP kernels.  There is no CPU fallback: if the built
library is missing, importing the solver raises.  The CPU restatement used to
check results lives in oracle/ and is test infrastructure only.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("GGMRES_LIB") or os.path.join(PKG_ROOT, "lib", "libggmres.so")

GG_OK, GG_NOT_CONVERGED = 0, 1
PRECOND_NONE, PRECOND_ILU0, PRECOND_ILUK, PRECOND_LU, PRECOND_SPLIT, PRECOND_USER, PRECOND_USER_SPLIT = range(7)
APPLY_MINV, APPLY_LEFT, APPLY_RIGHT, APPLY_START, APPLY_RHS = range(5)
SOLVE_SHARED_DEVICE = 0x1     # gg_options.flags: other solvers share the device (ggmres.h)
SOLVE_CGS2 = 0x2              # gg_options.flags: CGS2 orthogonalization (sharded solve only)

# every symbol include/ggmres.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "gg_abi_version", "gg_strerror", "gg_last_error", "gg_device_count", "gg_create",
    "gg_destroy", "gg_set_matrix", "gg_set_precond_none", "gg_set_precond_ilu0",
    "gg_set_precond_iluk", "gg_set_precond_lu", "gg_set_precond_split", "gg_precond_kind",
    "gg_uses_wavefront", "gg_solve", "gg_solve_device", "gg_get_history", "gg_spmv",
    "gg_precond_apply", "gg_time_spmv", "gg_time_precond", "gg_bytes_spmv",
    "gg_bytes_precond", "gg_profile_enable", "gg_profile_reset", "gg_profile_get",
    "gg_trace_precond", "gg_bytes_trsv", "gg_bytes_trsv_stream", "gg_transient", "gg_set_precond_ilu0_device",
    "gg_ilu0_device_values", "gg_set_precond_iluk_device", "gg_iluk_device_factors",
    "gg_transient_src", "gg_transient_set_taps", "gg_transient_get_taps", "gg_spmv_sliced", "gg_spmv_panels", "gg_spmv_rtile",
    "gg_transient_mna", "gg_set_division", "gg_division_active",
    "gg_trsv_kernel", "gg_mgs_kernel", "gg_set_precond_user", "gg_solve_device_f32",
    "gg_device_fingerprint", "gg_set_matrix_count", "gg_trsv_levels", "gg_layout", "gg_reduce_blocks",
    "gg_solve_batch_device", "gg_solve_batch", "gg_batch_engine", "gg_batch_history", "gg_transient_batch",
]
# gg_precond_fn: int (*)(void *ctx, int op, const float *in, float *out, int n), device arrays
PRECOND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_int)
DIV_EXACT, DIV_RCP, DIV_FMA = 0, 1, 2     # gg_div_mode
SRC_DC, SRC_PULSE, SRC_PWL = 0, 1, 2          # gg_src_kind
PROF_SPMV, PROF_PRECOND, PROF_MGS, PROF_TRSV_L, PROF_TRSV_U = range(5)
PROF_NKINDS = 5


class Options(ctypes.Structure):
    _fields_ = [("restart", ctypes.c_int), ("max_iter", ctypes.c_int),
                ("tol", ctypes.c_double), ("flags", ctypes.c_int)]


class Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("iters", ctypes.c_int),
                ("inner_iters", ctypes.c_int), ("restarts", ctypes.c_int),
                ("relres", ctypes.c_double), ("solve_ms", ctypes.c_double)]


class GGError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ggmres error {code}: {msg}")
        self.code = code


_lib = None
_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_D = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_VP = ctypes.c_void_p


def lib():
    """Load libggmres.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` "
                              "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.gg_strerror.restype = ctypes.c_char_p
        L.gg_last_error.restype = ctypes.c_char_p
        L.gg_create.argtypes = [ctypes.c_int, ctypes.POINTER(_VP)]
        L.gg_destroy.argtypes = [_VP]
        L.gg_set_matrix.argtypes = [_VP, ctypes.c_int, _I, _I, _D]
        for f in ("gg_set_precond_none", "gg_set_precond_ilu0", "gg_precond_kind",
                  "gg_uses_wavefront", "gg_spmv_sliced", "gg_set_precond_ilu0_device", "gg_spmv_panels",
                  "gg_spmv_rtile"):
            getattr(L, f).argtypes = [_VP]
        L.gg_set_precond_iluk.argtypes = [_VP, ctypes.c_int]
        L.gg_set_division.argtypes = [_VP, ctypes.c_int]
        L.gg_division_active.argtypes = [_VP, ctypes.c_int]
        L.gg_trsv_kernel.argtypes = [_VP, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.gg_mgs_kernel.argtypes = [_VP, ctypes.c_char_p, ctypes.c_int]
        L.gg_set_precond_iluk_device.argtypes = [_VP, ctypes.c_int]
        _PI, _PD = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)
        L.gg_iluk_device_factors.argtypes = [_VP, ctypes.c_int, _I, ctypes.POINTER(_PI), ctypes.POINTER(_PD),
                                             _I, ctypes.POINTER(_PI), ctypes.POINTER(_PD), _PD]
        L.gg_ilu0_device_values.argtypes = [_VP, _D, ctypes.POINTER(ctypes.c_double)]
        L.gg_set_precond_lu.argtypes = [_VP, _I, _I, _D, _I, _I, _D]
        L.gg_set_precond_split.argtypes = [_VP, _I, _I, _D, _I, _I, _D, _D, _I, _I, _D, _D]
        L.gg_set_precond_user.argtypes = [_VP, ctypes.c_int, PRECOND_FN, ctypes.c_void_p]
        L.gg_solve_device_f32.argtypes = [_VP, _VP, _VP, ctypes.POINTER(Options), ctypes.POINTER(Result)]
        L.gg_device_fingerprint.argtypes = [ctypes.POINTER(_VP), ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_ulonglong)]
        L.gg_set_matrix_count.restype = ctypes.c_longlong
        L.gg_trsv_levels.argtypes = [_VP, ctypes.c_int]
        L.gg_solve.argtypes = [_VP, _D, _D, ctypes.POINTER(Options), ctypes.POINTER(Result)]
        L.gg_solve_device.argtypes = [_VP, _VP, _VP, ctypes.POINTER(Options),
                                      ctypes.POINTER(Result)]
        L.gg_get_history.argtypes = [_VP, ctypes.c_void_p, ctypes.c_int]
        L.gg_transient_src.argtypes = [_VP, ctypes.c_int, ctypes.c_double, _D, ctypes.c_int, _I, _I, _I, _D,
                                       ctypes.c_int, _I, _D, ctypes.POINTER(Options), _D,
                                       ctypes.POINTER(ctypes.c_int)]
        L.gg_transient.argtypes = [_VP, ctypes.c_int, ctypes.c_double, _D, ctypes.c_int, _I, _D,
                                   ctypes.c_int, _I, _D, ctypes.POINTER(Options), _D,
                                   ctypes.POINTER(ctypes.c_int)]
        L.gg_transient_mna.argtypes = [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_double, _VP, _VP, _VP,
                                       ctypes.c_int, _I, _I, _D, _I, _I, _D, ctypes.c_int, _I, _D,
                                       ctypes.POINTER(Options), _D, ctypes.POINTER(ctypes.c_int)]
        L.gg_spmv.argtypes = [_VP, _D, _D]
        L.gg_precond_apply.argtypes = [_VP, ctypes.c_int, _D, _D]
        L.gg_time_spmv.argtypes = [_VP, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double)]
        L.gg_time_precond.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.gg_trace_precond.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong),
                                       ctypes.c_longlong, ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)]
        L.gg_bytes_spmv.argtypes = [_VP]
        L.gg_bytes_spmv.restype = ctypes.c_double
        L.gg_bytes_precond.argtypes = [_VP]
        L.gg_bytes_precond.restype = ctypes.c_double
        L.gg_bytes_trsv.argtypes = [_VP, ctypes.c_int]
        L.gg_bytes_trsv.restype = ctypes.c_double
        L.gg_bytes_trsv_stream.argtypes = [_VP, ctypes.c_int]
        L.gg_bytes_trsv_stream.restype = ctypes.c_double
        L.gg_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.gg_layout.argtypes = [_VP, ctypes.c_void_p, ctypes.c_longlong]
        L.gg_layout.restype = ctypes.c_longlong
        L.gg_reduce_blocks.argtypes = [_VP, ctypes.POINTER(ctypes.c_int)]
        L.gg_solve_batch_device.argtypes = [_VP, ctypes.c_int, _VP, ctypes.c_longlong, _VP, ctypes.c_longlong,
                                            ctypes.POINTER(Options), ctypes.POINTER(Result)]
        L.gg_solve_batch.argtypes = [_VP, ctypes.c_int, _D, ctypes.c_longlong, _D, ctypes.c_longlong,
                                     ctypes.POINTER(Options), ctypes.POINTER(Result)]
        L.gg_batch_engine.argtypes = [_VP]
        L.gg_batch_history.argtypes = [_VP, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong]
        L.gg_batch_history.restype = ctypes.c_longlong
        L.gg_transient_batch.argtypes = [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_double, _D, _I, _I, _I, _I, _D,
                                         ctypes.c_int, _I, _D, ctypes.POINTER(Options), _D, _I]
        L.gg_profile_enable.argtypes = [_VP, ctypes.c_int]
        L.gg_profile_reset.argtypes = [_VP]
        L.gg_profile_get.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def _check(rc, allow_nc=False):
    if rc < 0 or (rc == GG_NOT_CONVERGED and not allow_nc):
        raise GGError(rc, lib().gg_last_error().decode())
    return rc


def _csr_arrays(M):
    """scipy matrix / oracle CSR tuple -> (n, rp, ci, v) contiguous."""
    if hasattr(M, "tocsr"):
        M = M.tocsr()
        return (M.shape[0], np.ascontiguousarray(M.indptr, np.int32),
                np.ascontiguousarray(M.indices, np.int32), np.ascontiguousarray(M.data, np.float64))
    n, rp, ci, v = M
    return (n, np.ascontiguousarray(rp, np.int32), np.ascontiguousarray(ci, np.int32),
            np.ascontiguousarray(v, np.float64))


class Solver:
    """One solver on one GPU (handle of the C ABI)."""

    def __init__(self, device=0):
        h = _VP()
        _check(lib().gg_create(int(device), ctypes.byref(h)))
        self.h = h
        self.n = 0
        self.nnz = 0

    def close(self):
        if self.h:
            lib().gg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setup -----------------------------------------------------------
    def set_matrix(self, A):
        n, rp, ci, v = _csr_arrays(A)
        self.n = n
        self.nnz = int(rp[n])
        _check(lib().gg_set_matrix(self.h, n, rp, ci, v))

    def set_precond_none(self):
        _check(lib().gg_set_precond_none(self.h))

    def set_precond_ilu0(self):
        _check(lib().gg_set_precond_ilu0(self.h))

    def set_precond_ilu0_device(self):
        """ILU(0) factored on the GPU (bit-identical factors to set_precond_ilu0)."""
        _check(lib().gg_set_precond_ilu0_device(self.h))

    def ilu0_device_values(self):
        """(factored values in A's CSR order before the drop/split, device ms)."""
        out = np.zeros(self.nnz)
        ms = ctypes.c_double()
        _check(lib().gg_ilu0_device_values(self.h, out, ctypes.byref(ms)))
        return out, ms.value

    def set_precond_iluk(self, level):
        _check(lib().gg_set_precond_iluk(self.h, int(level)))

    def set_precond_iluk_device(self, level):
        """ILU(k) with the numeric phase on the GPU (bit-identical factors)."""
        _check(lib().gg_set_precond_iluk_device(self.h, int(level)))

    def iluk_device_factors(self, level):
        """((L rp, ci, v), (U rp, ci, v), device ms) of the device ILU(k)."""
        n = self.n
        lrp = np.zeros(n + 1, np.int32)
        urp = np.zeros(n + 1, np.int32)
        PI, PD = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)
        lci, lv, uci, uv = PI(), PD(), PI(), PD()
        ms = ctypes.c_double()
        _check(lib().gg_iluk_device_factors(self.h, int(level), lrp, ctypes.byref(lci), ctypes.byref(lv),
                                            urp, ctypes.byref(uci), ctypes.byref(uv), ctypes.byref(ms)))
        out = []
        for rp, ci, v in ((lrp, lci, lv), (urp, uci, uv)):
            nz = int(rp[n])
            c = np.ctypeslib.as_array(ci, shape=(max(nz, 1),))[:nz].copy()
            x = np.ctypeslib.as_array(v, shape=(max(nz, 1),))[:nz].copy()
            lib().gg_host_free(ctypes.cast(ci, ctypes.c_void_p))
            lib().gg_host_free(ctypes.cast(v, ctypes.c_void_p))
            out.append((rp, c, x))
        return out[0], out[1], ms.value

    def set_precond_lu(self, L, U):
        _, lrp, lci, lv = _csr_arrays(L)
        _, urp, uci, uv = _csr_arrays(U)
        _check(lib().gg_set_precond_lu(self.h, lrp, lci, lv, urp, uci, uv))

    def set_precond_split(self, L, U, middle, perm_row, perm_col, lscale, rscale):
        _, lrp, lci, lv = _csr_arrays(L)
        _, urp, uci, uv = _csr_arrays(U)
        f = lambda a: np.ascontiguousarray(a, np.float64)
        i = lambda a: np.ascontiguousarray(a, np.int32)
        _check(lib().gg_set_precond_split(self.h, lrp, lci, lv, urp, uci, uv, f(middle),
                                          i(perm_row), i(perm_col), f(lscale), f(rscale)))

    def set_precond_user(self, fn, split=False):
        """A caller-supplied preconditioner (the reference's Preconditioner
        plug-in): fn(op, in_ptr, out_ptr, n) -> int works on DEVICE arrays of n
        float32 (e.g. wrapped with torch); op is APPLY_MINV (split False) or
        APPLY_LEFT / RIGHT / START / RHS (split True).  Kept alive on the solver.
        An exception raised by fn is reported to the solver as status -1 (a
        ctypes callback that raises would return 0, i.e. success) and kept in
        self.user_exc."""
        self.user_exc = None

        def call(ctx, op, i, o, n):
            try:
                return int(fn(op, i, o, n))
            except BaseException as e:          # noqa: BLE001 -- must not cross the C frame
                self.user_exc = e
                return -1
        self._ufn = PRECOND_FN(call)
        _check(lib().gg_set_precond_user(self.h, 1 if split else 0, self._ufn, None))

    def set_division(self, mode):
        """DIV_EXACT (x = RN(acc/d), the default), DIV_RCP (x = RN(acc * RN(1/d))
        on the wavefront triangular solves) or DIV_FMA (rows as two fused
        multiply-adds, U pre-scaled by RN(1/d), on unskewed 2D-grid wavefronts;
        DIV_RCP elsewhere); both tolerance parity -- ggmres.h"""
        _check(lib().gg_set_division(self.h, int(mode)))

    def division_active(self, which):
        """the division triangle `which` (0 = L / Ml, 1 = U / Mr) runs with"""
        return _check(lib().gg_division_active(self.h, int(which)), allow_nc=True)

    def trsv_levels(self, which):
        """dependency chain of triangle `which`: levels (dataflow solve) or wavefront steps"""
        return _check(lib().gg_trsv_levels(self.h, int(which)), allow_nc=True)

    def trsv_kernel(self, which):
        """rocprofv3 name of the kernel running triangle `which` (0 = L, 1 = U)"""
        buf = ctypes.create_string_buffer(256)
        _check(lib().gg_trsv_kernel(self.h, int(which), buf, 256))
        return buf.value.decode()

    def mgs_kernel(self):
        """rocprofv3 name of the last solve's one-launch orthogonalization kernel
        ('' = the per-step kernels)"""
        buf = ctypes.create_string_buffer(256)
        _check(lib().gg_mgs_kernel(self.h, buf, 256))
        return buf.value.decode()

    @property
    def uses_wavefront(self):
        return bool(lib().gg_uses_wavefront(self.h))

    @property
    def spmv_sliced(self):
        """the matrix takes the sliced-ELL SpMV (else CSR-stream)"""
        return bool(lib().gg_spmv_sliced(self.h))

    @property
    def spmv_panels(self):
        """column panels y = A x runs over (k_spmv_panel), 0 = none"""
        return int(lib().gg_spmv_panels(self.h))

    @property
    def spmv_rtile(self):
        """row blocks of the one-launch panel SpMV (k_spmv_rtile), 0 = panel-major launches / none"""
        return int(lib().gg_spmv_rtile(self.h))

    # ---- solve -------------------------------------------------------------
    def solve(self, b, x0=None, restart=30, max_iter=3000, tol=1e-10, flags=0):
        b = np.ascontiguousarray(b, np.float64)
        x = np.zeros(self.n) if x0 is None else np.array(x0, np.float64, copy=True)
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        r = Result()
        rc = _check(lib().gg_solve(self.h, b, x, ctypes.byref(o), ctypes.byref(r)), allow_nc=True)
        return dict(ret=rc, x=x, iters=r.iters, inner=r.inner_iters, restarts=r.restarts,
                    relres=r.relres, solve_ms=r.solve_ms, hist=self.history())

    def solve_device(self, b_ptr, x_ptr, restart=30, max_iter=3000, tol=1e-10, flags=0):
        """b_ptr / x_ptr: device addresses (e.g. torch tensor .data_ptr()), natural order."""
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        r = Result()
        rc = _check(lib().gg_solve_device(self.h, _VP(b_ptr), _VP(x_ptr), ctypes.byref(o),
                                          ctypes.byref(r)), allow_nc=True)
        return dict(ret=rc, iters=r.iters, inner=r.inner_iters, restarts=r.restarts,
                    relres=r.relres, solve_ms=r.solve_ms)

    # ---- many right-hand sides (gg_solve_batch*, batch.hip) -----------------
    @property
    def batch_engine(self):
        """True when gg_solve_batch* runs batched launches (else scenario by scenario)"""
        return bool(_check(lib().gg_batch_engine(self.h), allow_nc=True))

    @staticmethod
    def _batch_out(rc, res):
        return dict(ret=rc, iters=[r.iters for r in res], inner=[r.inner_iters for r in res],
                    restarts=[r.restarts for r in res], relres=[r.relres for r in res],
                    status=[r.status for r in res], solve_ms=res[0].solve_ms if len(res) else 0.0)

    def solve_batch(self, B, X0=None, restart=30, max_iter=3000, tol=1e-10):
        """nrhs independent solves A x_q = b_q (rows of B), batched; returns
        dict(x [nrhs, n], iters / inner / restarts / relres / status per
        scenario, hist = per-scenario histories)."""
        B = np.ascontiguousarray(np.atleast_2d(B), np.float64)
        S, n = B.shape
        X = np.zeros((S, n)) if X0 is None else np.array(np.atleast_2d(X0), np.float64, copy=True, order="C")
        o = Options(int(restart), int(max_iter), float(tol), 0)
        res = (Result * S)()
        rc = _check(lib().gg_solve_batch(self.h, S, B.reshape(-1), n, X.reshape(-1), n, ctypes.byref(o), res),
                    allow_nc=True)
        out = self._batch_out(rc, res)
        out["x"] = X
        out["hist"] = [self.batch_history(q) for q in range(S)]
        return out

    def solve_batch_device(self, b_ptr, x_ptr, nrhs, ld=None, restart=30, max_iter=3000, tol=1e-10):
        """device addresses of nrhs right-hand sides / solutions, leading dimension ld (default n)"""
        ld = self.n if ld is None else int(ld)
        o = Options(int(restart), int(max_iter), float(tol), 0)
        res = (Result * int(nrhs))()
        rc = _check(lib().gg_solve_batch_device(self.h, int(nrhs), _VP(b_ptr), ld, _VP(x_ptr), ld,
                                                ctypes.byref(o), res), allow_nc=True)
        return self._batch_out(rc, res)

    def batch_history(self, q):
        """scenario q's residual history of the last batched solve (empty when
        the scenarios ran one by one: see history() after each)"""
        n = int(lib().gg_batch_history(self.h, int(q), None, 0))
        if n < 0:
            return np.zeros(0)
        out = np.zeros(n)
        lib().gg_batch_history(self.h, int(q), out.ctypes.data, n)
        return out

    def transient_batch(self, nsteps, h, cdiag, scenarios, ports, X0, restart=32, max_iter=10000, tol=1e-7):
        """gg_transient_batch: scenarios = [(src_node, sources), ...] with sources
        = [(kind, params), ...] (as transient_src) or a PULSE parameter array
        (n_src x 7); X0 [nrhs, n].  Returns dict(x [nrhs, n], ports [nrhs, nport,
        nsteps+1], iters_total [nrhs], ret)."""
        S = len(scenarios)
        X = np.array(np.atleast_2d(X0), np.float64, copy=True, order="C")
        assert X.shape == (S, self.n)
        nodes, kinds, lens, datas, off = [], [], [], [], [0]
        for src_node, sources in scenarios:
            if not isinstance(sources, (list, tuple)):
                sources = [(SRC_PULSE, q) for q in np.asarray(sources, np.float64).reshape(-1, 7)]
            nodes.append(np.asarray(src_node, np.int32))
            kinds += [k for k, _ in sources]
            lens += [len(q) for _, q in sources]
            datas += [np.asarray(q, np.float64) for _, q in sources]
            off.append(off[-1] + len(sources))
        node = np.concatenate(nodes).astype(np.int32) if off[-1] else np.zeros(1, np.int32)
        kind = np.array(kinds or [0], np.int32)
        ptr = np.zeros(off[-1] + 1, np.int32)
        ptr[1:] = np.cumsum(lens) if lens else []
        data = np.concatenate(datas) if datas else np.zeros(1)
        ports = np.ascontiguousarray(ports, np.int32)
        pv = np.zeros(max(S * len(ports) * (nsteps + 1), 1))
        tot = np.zeros(S, np.int32)
        o = Options(int(restart), int(max_iter), float(tol), 0)
        one = np.zeros(1, np.int32)
        rc = _check(lib().gg_transient_batch(self.h, S, int(nsteps), float(h), np.ascontiguousarray(cdiag, np.float64),
                                             np.array(off, np.int32), node, kind, ptr, data, len(ports),
                                             ports if len(ports) else one, X.reshape(-1), ctypes.byref(o), pv, tot),
                    allow_nc=True)
        return dict(x=X, ports=pv[: S * len(ports) * (nsteps + 1)].reshape(S, len(ports), nsteps + 1),
                    iters_total=[int(t) for t in tot], ret=rc)

    def transient(self, nsteps, h, cdiag, src_node, pulse, ports, x0, restart=32,
                  max_iter=10000, tol=1e-7, flags=0):
        """Backward-Euler loop on the device (gg_transient): returns dict(x, ports
        [nport, nsteps+1], iters_total, ret)."""
        n = self.n
        x = np.array(x0, np.float64, copy=True)
        src_node = np.ascontiguousarray(src_node, np.int32)
        pulse = np.ascontiguousarray(pulse, np.float64).reshape(-1)
        ports = np.ascontiguousarray(ports, np.int32)
        pv = np.zeros(max(len(ports), 1) * (nsteps + 1))
        tot = ctypes.c_int()
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        rc = _check(lib().gg_transient(self.h, int(nsteps), float(h),
                                       np.ascontiguousarray(cdiag, np.float64), len(src_node),
                                       src_node if len(src_node) else np.zeros(1, np.int32),
                                       pulse if pulse.size else np.zeros(7), len(ports),
                                       ports if len(ports) else np.zeros(1, np.int32), x,
                                       ctypes.byref(o), pv, ctypes.byref(tot)), allow_nc=True)
        return dict(x=x, ports=pv[: len(ports) * (nsteps + 1)].reshape(len(ports), nsteps + 1),
                    iters_total=tot.value, ret=rc)

    def transient_src(self, nsteps, h, cdiag, src_node, sources, ports, x0, restart=32,
                      max_iter=10000, tol=1e-7, flags=0):
        """gg_transient_src: sources = [(kind, params), ...] (SRC_DC / SRC_PULSE /
        SRC_PWL); returns dict(x, ports [nport, nsteps+1], iters_total, ret)."""
        n = self.n
        x = np.array(x0, np.float64, copy=True)
        src_node = np.ascontiguousarray(src_node, np.int32)
        kind = np.array([k for k, _ in sources], np.int32)
        ptr = np.zeros(len(sources) + 1, np.int32)
        ptr[1:] = np.cumsum([len(q) for _, q in sources])
        data = np.concatenate([np.asarray(q, np.float64) for _, q in sources]) if sources else np.zeros(1)
        ports = np.ascontiguousarray(ports, np.int32)
        pv = np.zeros(max(len(ports), 1) * (nsteps + 1))
        tot = ctypes.c_int()
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        one = np.zeros(1, np.int32)
        rc = _check(lib().gg_transient_src(self.h, int(nsteps), float(h), np.ascontiguousarray(cdiag, np.float64),
                                           len(src_node), src_node if len(src_node) else one,
                                           kind if len(kind) else one, ptr, data, len(ports),
                                           ports if len(ports) else one, x, ctypes.byref(o), pv,
                                           ctypes.byref(tot)), allow_nc=True)
        return dict(x=x, ports=pv[: len(ports) * (nsteps + 1)].reshape(len(ports), nsteps + 1),
                    iters_total=tot.value, ret=rc)

    def transient_mna(self, it0, nsteps, h, R, B, sources, ports, x0, restart=32, max_iter=10000,
                      tol=1e-7, flags=0):
        """gg_transient_mna: w = B u(it h) + R x per step, it = it0 .. it0+nsteps-1;
        R (n x n) and B (n x nsrc) scipy sparse (R None = 0); sources as
        transient_src.  Returns dict(x, ports [nport, nsteps+1], iters_total, ret)."""
        import scipy.sparse as sp
        x = np.array(x0, np.float64, copy=True)
        n = len(x)
        Bc = sp.csr_matrix(B)
        Bc.sort_indices()
        keep = []
        if R is not None:
            Rc = sp.csr_matrix(R)
            Rc.sort_indices()
            rp = np.ascontiguousarray(Rc.indptr, np.int32)
            ri = np.ascontiguousarray(Rc.indices, np.int32) if Rc.nnz else np.zeros(1, np.int32)
            rv = np.ascontiguousarray(Rc.data, np.float64) if Rc.nnz else np.zeros(1)
            keep = [rp, ri, rv]
            rargs = [rp.ctypes.data, ri.ctypes.data, rv.ctypes.data]
        else:
            rargs = [None, None, None]
        bp = np.ascontiguousarray(Bc.indptr, np.int32)
        bi = np.ascontiguousarray(Bc.indices, np.int32) if Bc.nnz else np.zeros(1, np.int32)
        bv = np.ascontiguousarray(Bc.data, np.float64) if Bc.nnz else np.zeros(1)
        kind = np.array([k for k, _ in sources] or [0], np.int32)
        ptr = np.zeros(len(sources) + 1, np.int32)
        ptr[1:] = np.cumsum([len(q) for _, q in sources])
        data = np.concatenate([np.asarray(q, np.float64) for _, q in sources]) if sources else np.zeros(1)
        ports = np.ascontiguousarray(ports, np.int32)
        pv = np.zeros(max(len(ports), 1) * (nsteps + 1))
        tot = ctypes.c_int()
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        rc = _check(lib().gg_transient_mna(self.h, int(it0), int(nsteps), float(h), *rargs, len(sources),
                                           bp, bi, bv, kind, ptr, data, len(ports),
                                           ports if len(ports) else np.zeros(1, np.int32), x,
                                           ctypes.byref(o), pv, ctypes.byref(tot)), allow_nc=True)
        del keep
        return dict(x=x, ports=pv[: len(ports) * (nsteps + 1)].reshape(len(ports), nsteps + 1),
                    iters_total=tot.value, ret=rc)

    def set_taps(self, tap_node):
        """tap nodes whose max / min / avg / IR drop the next transient runs track"""
        t = np.ascontiguousarray(tap_node, np.int32)
        _check(lib().gg_transient_set_taps(self.h, len(t), t.ctypes.data_as(ctypes.c_void_p)))
        self._ntap = len(t)

    def get_taps(self):
        """(max, min, avg, ir) of the tap nodes over the last transient run."""
        out = [np.zeros(getattr(self, "_ntap", 0)) for _ in range(4)]
        _check(lib().gg_transient_get_taps(self.h, *[o.ctypes.data_as(ctypes.c_void_p) for o in out]))
        return tuple(out)

    def history(self):
        n = lib().gg_get_history(self.h, None, 0)
        out = np.zeros(max(n, 1))
        lib().gg_get_history(self.h, out.ctypes.data_as(ctypes.c_void_p), n)
        return out[:n]

    # ---- single operators ----------------------------------------------------
    def spmv(self, x):
        y = np.zeros(self.n)
        _check(lib().gg_spmv(self.h, np.ascontiguousarray(x, np.float64), y))
        return y

    def precond_apply(self, op, v):
        out = np.zeros(self.n)
        _check(lib().gg_precond_apply(self.h, int(op), np.ascontiguousarray(v, np.float64), out))
        return out

    def time_spmv(self, reps=50, nrot=4):
        ms = ctypes.c_double()
        _check(lib().gg_time_spmv(self.h, int(reps), int(nrot), ctypes.byref(ms)))
        return ms.value

    def trace_precond(self, which=0, cap=1 << 20):
        """Per-band batch-start timestamps (100 MHz clock) of one wavefront
        triangular solve: array [nbands, 3*nbatch+8] (layout in ggmres.h)."""
        import numpy as np
        buf = (ctypes.c_longlong * cap)()
        nb, nbt = ctypes.c_int(), ctypes.c_int()
        _check(lib().gg_trace_precond(self.h, int(which), buf, cap, ctypes.byref(nb),
                                      ctypes.byref(nbt)))
        a = np.ctypeslib.as_array(buf)[: nb.value * (3 * nbt.value + 8)].copy()
        return a.reshape(nb.value, 3 * nbt.value + 8)

    def trace_tiles(self, which=0):
        """3D tile wavefront (k_trsv_tile3d) diagnostics of one triangular solve:
        array [tiles, 8 + 5 nbatch] per tile (band = K*NJ + J): compute start /
        end (100 MHz realtime), workgroup, boundary poll retries, retry cycles,
        realtime after batch 0, loader start; per batch: compute start, writer
        publication, boundary values seen, loader landed, compute end."""
        import numpy as np
        cap = 1 << 22
        buf = (ctypes.c_longlong * cap)()
        nb, nbt = ctypes.c_int(), ctypes.c_int()
        _check(lib().gg_trace_precond(self.h, int(which), buf, cap, ctypes.byref(nb),
                                      ctypes.byref(nbt)))
        w = 8 + 5 * nbt.value
        return np.ctypeslib.as_array(buf)[: nb.value * w].copy().reshape(nb.value, w)

    def time_precond(self, reps=20):
        ms = ctypes.c_double()
        _check(lib().gg_time_precond(self.h, int(reps), ctypes.byref(ms)))
        return ms.value

    def profile(self, on=True, kinds=None):
        """Time kernel families inside solves: kinds = iterable of PROF_* (default all)."""
        mask = 0
        if on:
            mask = (1 << PROF_NKINDS) - 1 if kinds is None else sum(1 << int(k) for k in set(kinds))
        _check(lib().gg_profile_enable(self.h, mask))
        _check(lib().gg_profile_reset(self.h))

    def layout(self):
        """(lay2nat, G): the natural row at each slot of the solver's vector space
        (-1 = padding) and the reduction grid of its dots -- the order the
        order-matched oracle needs (oracle.set_dot_order)."""
        P = int(lib().gg_layout(self.h, None, 0))
        if P < 0:
            _check(P)
        out = np.empty(P, np.int64)
        lib().gg_layout(self.h, out.ctypes.data, P)
        G = ctypes.c_int()
        _check(lib().gg_reduce_blocks(self.h, ctypes.byref(G)))     # the solver's own s->G
        return out, G.value

    def profile_select(self, kinds):
        """Switch the timed families to `kinds` WITHOUT clearing what was
        accumulated (bench.py rotates one bracketed family per timed solve)."""
        mask = sum(1 << int(k) for k in set(kinds))
        _check(lib().gg_profile_enable(self.h, mask))

    def profile_get(self, kind):
        """(launches, total_ms) of one kernel family over the profiled solves."""
        n, ms = ctypes.c_int(), ctypes.c_double()
        _check(lib().gg_profile_get(self.h, int(kind), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def bytes_spmv(self):
        return lib().gg_bytes_spmv(self.h)

    def bytes_precond(self):
        return lib().gg_bytes_precond(self.h)

    def bytes_trsv(self, which):
        """algorithmic bytes of one triangular solve (0 = L / Ml, 1 = U / Mr;
        SURVEY.md 8(d)'s CSR formulation)"""
        return lib().gg_bytes_trsv(self.h, int(which))

    def bytes_trsv_stream(self, which):
        """bytes the triangular solve's kernel itself streams (no index arrays on
        the wavefront)"""
        return lib().gg_bytes_trsv_stream(self.h, int(which))


def device_count():
    c = ctypes.c_int()
    _check(lib().gg_device_count(ctypes.byref(c)))
    return c.value
