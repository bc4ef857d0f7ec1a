"""CPU restatement of the SHARDED solve (TEST INFRASTRUCTURE ONLY).

It runs the decomposition the product's gpu-gmres_amd/csrc/dd.hip runs, on
the pieces the product's host code (gg_host_dd_*, csrc/host/dd_setup.cpp)
extracts, with serial fp64 arithmetic from oracle.c, and exchanges data
through a caller-supplied all-gather: in-process (all shards in one Python
process) or torch.distributed (gloo, one shard per process).  The tests
check it against the GLOBAL restatement on the arrow-permuted matrix
B = P A P^T (partition4 src/partition3.cpp:122-194, dd_form
src/form_dd.cpp:32-110):

  * SpMV and the ILU(0) apply are bit-identical to oracle.spmv(B, .) /
    oracle.lusolve(ilu0(B), .) -- the split of each row of
    LUSolve_ignoreZero (src/SpMV_compute.cpp:92-136) into "coupling terms
    first, then the own triangle" keeps the reference's operation order;
  * GMRES_leftILU0 (src/gmres.cu:566-717) restated with sharded dots (each
    shard's serial partial over its rows, partials summed in shard order)
    matches oracle.gmres_left on B to 1e-10 (the dot order differs).
"""
import numpy as np

from . import CSR, lib, spmv as _spmv


def csr(M):
    """scipy CSR -> oracle CSR keeping the entry order of every row (the
    pieces list their terms in the reference's summation order)"""
    if isinstance(M, CSR):
        return M
    return CSR(M.shape[0], np.ascontiguousarray(M.indptr, np.int32),
               np.ascontiguousarray(M.indices, np.int32), np.ascontiguousarray(M.data, np.float64))

_i32 = lambda a: np.ascontiguousarray(a, np.int32)
_f64 = lambda a: np.ascontiguousarray(a, np.float64)


def _tri(T, d, b, lower):
    T = csr(T)
    x = np.zeros(T.n)
    if T.n:
        lib().orc_canon_trsv(T.n, 1 if lower else 0, T.rp, T.ci, T.v, _f64(d), _f64(b), x)
    return x


def _sub(C, x, vin):
    C = csr(C)
    out = np.zeros(C.n)
    if C.n:
        lib().orc_sub_seq(C.n, C.rp, C.ci, C.v, _f64(x), _f64(vin), out)
    return out


class Shard:
    """Shard p's operators on local vectors [interior nI | separator nS | halo P*maxI]."""

    def __init__(self, piece, p, P, max_iface):
        self.s, self.p, self.P, self.maxI = piece, p, P, max_iface
        self.nI, self.nS = piece["nI"], piece["nS"]
        self.nloc = self.nI + self.nS
        self.A = csr(piece["A"])

    def local(self, vB):
        """this shard's rows of a vector in permuted (B) order, halo zeroed"""
        v = np.zeros(self.nloc + self.P * self.maxI)
        v[: self.nloc] = vB[self.s["rows"]]
        return v

    def pack(self, v):
        out = np.zeros(self.maxI)
        out[: len(self.s["iface"])] = v[self.s["iface"]]
        return out

    def dot_range(self):
        return self.nloc if self.p == 0 else self.nI


class Group:
    """The shards this process holds + the all-gather that connects all shards.
    allgather(list of per-local-shard arrays) -> list (length P) of arrays."""

    def __init__(self, shards, P, allgather):
        self.sh, self.P, self.ag = shards, P, allgather

    def halo(self, vs):
        if self.sh[0].maxI == 0:
            return
        parts = self.ag([s.pack(v) for s, v in zip(self.sh, vs)])
        h = np.concatenate(parts)
        for s, v in zip(self.sh, vs):
            v[s.nloc:] = h

    def spmv(self, xs):
        self.halo(xs)
        return [self._ext(s, _spmv(s.A, x)) for s, x in zip(self.sh, xs)]

    def resid(self, xs, bs):
        ys = self.spmv(xs)
        return [self._ext(s, b[: s.nloc] - y[: s.nloc]) for s, b, y in zip(self.sh, bs, ys)]

    def _ext(self, s, v):
        out = np.zeros(s.nloc + s.P * s.maxI)
        out[: s.nloc] = v[: s.nloc]
        return out

    def apply(self, ys):
        """(LU)^-1 of B's ILU(0), sharded (dd_setup.cpp module comment)"""
        t1 = []
        for s, y in zip(self.sh, ys):
            v = np.zeros(s.nloc + s.P * s.maxI)
            v[: s.nI] = _tri(s.s["LI"], s.s["dLI"], y[: s.nI], True)
            t1.append(v)
        self.halo(t1)
        out = []
        for s, y, v in zip(self.sh, ys, t1):
            nI = s.nI
            t2s = _sub(s.s["LSH"], v[s.nloc:], y[nI: s.nloc])
            ys_ = _tri(s.s["LS"], s.s["dLS"], t2s, True)
            xs_ = _tri(s.s["US"], s.s["dUS"], ys_, False)
            t2i = _sub(s.s["UIS"], xs_, v[:nI])
            xi = _tri(s.s["UI"], s.s["dUI"], t2i, False)
            o = np.zeros_like(v)
            o[:nI] = xi
            o[nI: s.nloc] = xs_
            out.append(o)
        return out

    def dot(self, a, b):
        parts = []
        for s, x, y in zip(self.sh, a, b):     # this shard's rows (separator on shard 0)
            k = s.dot_range()
            parts.append(np.array([float(np.dot(x[:k], y[:k]))]))
        allp = self.ag(parts)
        t = 0.0
        for v in allp:                           # shard order, identical on every shard
            t += float(v[0])
        return t


def gmres_left(g, bs, xs, m=30, max_iter=3000, tol=1e-10):
    """GMRES_leftILU0 (src/gmres.cu:566-717) on sharded vectors; mirrors
    oracle.c gmres_core (kind 0) operation for operation.  Returns dict like
    oracle.gmres_left (x as the list of local vectors)."""
    norm = lambda v: np.sqrt(g.dot(v, v))
    hist = []
    bb = g.apply(bs)
    normb = norm(bb)
    if normb == 0.0:
        normb = 1.0
    r = g.apply(g.resid(xs, bs))
    beta = norm(r)
    resid = beta / normb
    hist.append(resid)
    if resid <= tol:
        return dict(ret=0, x=xs, iters=0, relres=resid, hist=np.array(hist))
    H = np.zeros((m + 1, m))
    s = np.zeros(m + 1)
    cs = np.zeros(m + 1)
    sn = np.zeros(m + 1)
    j = 1

    def rot(dx, dy, c, sv):
        return c * dx + sv * dy, -sv * dx + c * dy

    def gen(dx, dy):
        if dy == 0.0:
            return 1.0, 0.0
        if abs(dy) > abs(dx):
            t = dx / dy
            sv = 1.0 / np.sqrt(1.0 + t * t)
            return t * sv, sv
        t = dy / dx
        c = 1.0 / np.sqrt(1.0 + t * t)
        return c, t * c

    def update(k, V):
        y = s[: k + 1].copy()
        for i in range(k, -1, -1):
            y[i] /= H[i, i]
            for jj in range(i - 1, -1, -1):
                y[jj] -= H[jj, i] * y[i]
        for q, x in enumerate(xs):
            for jj in range(k + 1):
                x[:] = x + V[jj][q] * y[jj]

    while j <= max_iter:
        V = [[(1.0 / beta) * v for v in r]]
        s[:] = 0.0
        s[0] = beta
        i = 0
        while i < m and j <= max_iter:
            w = g.apply(g.spmv(V[i]))
            for k in range(i + 1):
                h = g.dot(w, V[k])
                H[k, i] = h
                w = [(-h) * vk + wq for vk, wq in zip(V[k], w)]
            hn = norm(w)
            H[i + 1, i] = hn
            V.append([(1.0 / hn) * wq if hn != 0.0 else 0.0 * wq for wq in w])
            for k in range(i):
                H[k, i], H[k + 1, i] = rot(H[k, i], H[k + 1, i], cs[k], sn[k])
            cs[i], sn[i] = gen(H[i, i], H[i + 1, i])
            H[i, i], H[i + 1, i] = rot(H[i, i], H[i + 1, i], cs[i], sn[i])
            s[i], s[i + 1] = rot(s[i], s[i + 1], cs[i], sn[i])
            resid = abs(s[i + 1]) / normb
            hist.append(resid)
            if resid < tol:
                update(i, V)
                return dict(ret=0, x=xs, iters=j, relres=resid, hist=np.array(hist))
            i += 1
            j += 1
        update(i - 1, V)
        r = g.apply(g.resid(xs, bs))
        beta = norm(r)
        resid = beta / normb
        hist.append(resid)
        if resid < tol:
            return dict(ret=0, x=xs, iters=j, relres=resid, hist=np.array(hist))
    return dict(ret=1, x=xs, iters=max_iter, relres=resid, hist=np.array(hist))
