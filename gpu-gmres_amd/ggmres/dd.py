"""Sharded GMRES(m) + ILU(0) over P GPUs (include/ggmres_dd.h).

DD(nparts, device=0)                    all shards in this process on one GPU
DD(nparts, rank=r, uid=bytes, device=d) one shard per process (RCCL); uid from
                                        unique_id() on rank 0, broadcast by the caller
DD(nparts, rank=r, comm="ipc", device=d) one shard per process, device-initiated
                                        exchanges through hipIpc-mapped areas; then
                                        d.connect_ipc(allgather) with any host
                                        all-gather of bytes (e.g. torch.distributed)
DD(nparts, rank=r, comm="loopback")     timing only: shard r alone, every exchange the
                                        in-process all-gather over its own buffer (run a
                                        fixed iteration count: the values are not the system's)
"""
import ctypes

import numpy as np

from . import Options, Result, _check, _csr_arrays, lib

LOCAL, RCCL, IPC, LOOPBACK = 0, 1, 2, 3
ID_BYTES = 128
IPC_HANDLE_BYTES = 64
_VP = ctypes.c_void_p
_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_D = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_done = False

EXPORTS = ["gg_dd_unique_id", "gg_dd_create", "gg_dd_destroy", "gg_dd_comm_ranks",
           "gg_dd_ipc_handle", "gg_dd_ipc_connect",
           "gg_dd_set_system", "gg_dd_info", "gg_dd_xk_active",
           "gg_dd_perm", "gg_dd_dot_layout", "gg_dd_solve", "gg_dd_solve_device",
           "gg_dd_get_history", "gg_dd_spmv", "gg_dd_precond_apply", "gg_dd_set_division",
           "gg_dd_time_exchange", "gg_dd_profile_enable", "gg_dd_profile_reset", "gg_dd_profile_get",
           "gg_dd_bytes"]
# gg_dd_prof_kind (ggmres_dd.h)
PROF_SPMV, PROF_TRSV_L, PROF_SEP, PROF_TRSV_U, PROF_ORTH = range(5)
PROF_NAMES = ("spmv", "trsv_L", "separator", "trsv_U", "orthogonalization")


def _lib():
    global _done
    L = lib()
    if not _done:
        L.gg_dd_unique_id.argtypes = [ctypes.c_char_p]
        L.gg_dd_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_char_p, ctypes.POINTER(_VP)]
        L.gg_dd_destroy.argtypes = [_VP]
        L.gg_dd_ipc_handle.argtypes = [_VP, ctypes.c_char_p]
        L.gg_dd_ipc_connect.argtypes = [_VP, ctypes.c_char_p]
        L.gg_dd_comm_ranks.argtypes = [_VP, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.gg_dd_set_system.argtypes = [_VP, ctypes.c_int, _I, _I, _D, ctypes.c_int]
        L.gg_dd_info.argtypes = [_VP, _I]
        L.gg_dd_xk_active.argtypes = [_VP, ctypes.POINTER(ctypes.c_int)]
        L.gg_dd_perm.argtypes = [_VP, _I, _I]
        L.gg_dd_dot_layout.argtypes = [_VP, ctypes.c_int, _VP, ctypes.c_longlong,
                                       ctypes.POINTER(ctypes.c_int)]
        L.gg_dd_solve.argtypes = [_VP, _D, _D, ctypes.POINTER(Options), ctypes.POINTER(Result)]
        L.gg_dd_solve_device.argtypes = [_VP, _VP, _VP, ctypes.POINTER(Options),
                                         ctypes.POINTER(Result)]
        L.gg_dd_get_history.argtypes = [_VP, _VP, ctypes.c_int]
        L.gg_dd_spmv.argtypes = [_VP, _D, _D]
        L.gg_dd_precond_apply.argtypes = [_VP, _D, _D]
        L.gg_dd_set_division.argtypes = [_VP, ctypes.c_int]
        L.gg_dd_time_exchange.argtypes = [_VP, ctypes.c_longlong, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.gg_dd_profile_enable.argtypes = [_VP, ctypes.c_int]
        L.gg_dd_profile_reset.argtypes = [_VP]
        L.gg_dd_profile_get.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_double)]
        L.gg_dd_bytes.argtypes = [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        _done = True
    return L


def unique_id():
    buf = ctypes.create_string_buffer(ID_BYTES)
    _check(_lib().gg_dd_unique_id(buf))
    return buf.raw


class DD:
    def __init__(self, nparts, device=0, rank=None, uid=None, comm=None):
        h = _VP()
        kind = IPC if comm == "ipc" else LOOPBACK if comm == "loopback" else LOCAL if rank is None else RCCL
        if kind in (IPC, LOOPBACK) and rank is None:
            raise ValueError(f"dd: comm={comm!r} needs a rank")
        _check(_lib().gg_dd_create(int(device), int(nparts), kind, int(rank or 0),
                                   uid if uid is not None else None, ctypes.byref(h)))
        self.h, self.P, self.kind, self.rank = h, nparts, kind, rank
        self.n = 0

    def ipc_handle(self):
        """this rank's exchange-area handle (GG_DD_IPC)"""
        buf = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
        _check(_lib().gg_dd_ipc_handle(self.h, buf))
        return buf.raw

    def ipc_connect(self, handles):
        """every rank's handle, rank order: maps the peers' areas (collective)"""
        if len(handles) != self.P or any(len(x) != IPC_HANDLE_BYTES for x in handles):
            raise ValueError("dd: need nparts handles of IPC_HANDLE_BYTES")
        _check(_lib().gg_dd_ipc_connect(self.h, b"".join(handles)))

    def connect_ipc(self, allgather):
        """allgather(bytes) -> list of every rank's bytes (rank order)"""
        self.ipc_connect(list(allgather(self.ipc_handle())))

    def close(self):
        if self.h:
            _lib().gg_dd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def comm_ranks(self):
        """(ranks in the exchange, this process's rank): RCCL ncclCommCount, IPC the
        mapped areas (collective: every rank must call it), LOCAL (1, 0)"""
        c, r = ctypes.c_int(), ctypes.c_int()
        _check(_lib().gg_dd_comm_ranks(self.h, ctypes.byref(c), ctypes.byref(r)))
        return c.value, r.value

    def set_system(self, A, method=1):
        n, rp, ci, v = _csr_arrays(A)
        self.n = n
        _check(_lib().gg_dd_set_system(self.h, n, rp, ci, v, int(method)))

    def info(self):
        a = np.zeros(10, np.int32)
        _check(_lib().gg_dd_info(self.h, a))
        keys = ["n", "nparts", "nsep", "max_iface", "n_interior", "wave_interior", "wave_separator",
                "local_len", "shards_here", "halo_doubles"]
        out = dict(zip(keys, (int(x) for x in a)))
        on = ctypes.c_int()
        _check(_lib().gg_dd_xk_active(self.h, ctypes.byref(on)))
        out["cgs2_in_kernel_exchange"] = on.value
        return out

    def perm(self):
        pinv = np.zeros(self.n, np.int32)
        q = np.zeros(self.n, np.int32)
        _check(_lib().gg_dd_perm(self.h, pinv, q))
        return pinv, q

    def dot_layout(self, part):
        G = ctypes.c_int()
        ln = _check(_lib().gg_dd_dot_layout(self.h, int(part), None, 0, ctypes.byref(G)), True)
        out = np.zeros(max(ln, 1), np.int64)
        _lib().gg_dd_dot_layout(self.h, int(part), out.ctypes.data, ln, ctypes.byref(G))
        return out[:ln], G.value

    def solve(self, b, x0=None, restart=30, max_iter=3000, tol=1e-10, flags=0):
        """flags: ggmres.SOLVE_CGS2 for the three-all-gather orthogonalization"""
        b = np.ascontiguousarray(b, np.float64)
        x = np.zeros(self.n) if x0 is None else np.array(x0, np.float64, copy=True)
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        r = Result()
        rc = _check(_lib().gg_dd_solve(self.h, b, x, ctypes.byref(o), ctypes.byref(r)), allow_nc=True)
        return dict(ret=rc, x=x, iters=r.iters, inner=r.inner_iters, restarts=r.restarts,
                    relres=r.relres, solve_ms=r.solve_ms, hist=self.history())

    def solve_device(self, b_ptr, x_ptr, restart=30, max_iter=3000, tol=1e-10, flags=0):
        o = Options(int(restart), int(max_iter), float(tol), int(flags))
        r = Result()
        rc = _check(_lib().gg_dd_solve_device(self.h, _VP(b_ptr), _VP(x_ptr), ctypes.byref(o),
                                              ctypes.byref(r)), allow_nc=True)
        return dict(ret=rc, iters=r.iters, inner=r.inner_iters, restarts=r.restarts,
                    relres=r.relres, solve_ms=r.solve_ms)

    def history(self):
        n = _lib().gg_dd_get_history(self.h, None, 0)
        out = np.zeros(max(n, 1))
        _lib().gg_dd_get_history(self.h, out.ctypes.data, n)
        return out[:n]

    def spmv(self, x, y=None):
        y = np.zeros(self.n) if y is None else np.array(y, np.float64, copy=True)
        _check(_lib().gg_dd_spmv(self.h, np.ascontiguousarray(x, np.float64), y))
        return y

    def set_division(self, mode):
        """ggmres.DIV_EXACT / DIV_RCP / DIV_FMA for the shards' wavefront triangular solves"""
        _check(_lib().gg_dd_set_division(self.h, int(mode)))

    def profile(self, on=True, kinds=None):
        """in-solve timing of the families (PROF_*) of every inner iteration"""
        mask = 0
        if on:
            mask = (1 << len(PROF_NAMES)) - 1 if kinds is None else sum(1 << k for k in kinds)
        _check(_lib().gg_dd_profile_reset(self.h))
        _check(_lib().gg_dd_profile_enable(self.h, mask))

    def profile_get(self, kind):
        n, ms = ctypes.c_int(), ctypes.c_double()
        _check(_lib().gg_dd_profile_get(self.h, int(kind), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def bytes(self, kind):
        """algorithmic bytes of one launch of family kind (PROF_SPMV / _TRSV_L / _TRSV_U), this process's shards"""
        b = ctypes.c_double()
        _check(_lib().gg_dd_bytes(self.h, int(kind), ctypes.byref(b)))
        return b.value

    def time_exchange(self, cnt, reps=200):
        """average microseconds of one all-gather of cnt doubles per shard"""
        us = ctypes.c_double()
        _check(_lib().gg_dd_time_exchange(self.h, int(cnt), int(reps), ctypes.byref(us)))
        return us.value

    def precond_apply(self, v, out=None):
        out = np.zeros(self.n) if out is None else np.array(out, np.float64, copy=True)
        _check(_lib().gg_dd_precond_apply(self.h, np.ascontiguousarray(v, np.float64), out))
        return out
