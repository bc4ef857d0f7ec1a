"""Test infrastructure only: restatement of the reference's domain-decomposition
setup and Matrix Market reader, used by tests/test_partition.py to check the
product's host code (gpu-gmres_amd/csrc/host/partition.cpp, mtx.cpp).

partition4_adjust  src/partition3.cpp:149-193 (cut-edge endpoints to the
                   separator part, part sizes, pinv / q)
dd_blocks          src/form_dd.cpp:32-110 (As, E, F, At of the permuted matrix)
read_mtx           src_thermal/SpMV_gen.cpp:93-187 (readSparseMatrix, row-major)

METIS_PartGraphRecursive itself is not restated (METIS 4/5 is not vendored in
the reference and not installed); the base partition is an input here.
"""
import numpy as np


def node_graph(rp, ci, n):
    """symmetrized pattern without the diagonal: list of neighbour sets"""
    nb = [set() for _ in range(n)]
    for r in range(n):
        for k in range(rp[r], rp[r + 1]):
            c = int(ci[k])
            if c != r:
                nb[r].add(c)
                nb[c].add(r)
    return [sorted(s) for s in nb]


def partition4_adjust(rp, ci, n, nparts, base):
    """base: node -> part in 0..nparts-1 (METIS' output).  Returns node_part,
    part_size, pinv, q exactly as partition4 forms them."""
    nb = node_graph(rp, ci, n)
    node_part = np.array(base, np.int64)
    top = set()
    for j in range(n):
        for w in nb[j]:
            if node_part[w] != node_part[j]:
                top.add(w)
                top.add(j)
    for v in top:
        node_part[v] = nparts
    part_size = np.bincount(node_part, minlength=nparts + 1)
    begin = np.concatenate([[0], np.cumsum(part_size)])
    cur = np.zeros(nparts + 1, np.int64)
    pinv = np.zeros(n, np.int64)
    q = np.zeros(n, np.int64)
    for j in range(n):
        p = node_part[j]
        pinv[j] = begin[p] + cur[p]
        q[begin[p] + cur[p]] = j
        cur[p] += 1
    return node_part, part_size, pinv, q


def color_separator(rp, ci, n, nparts, node_part, pinv, q):
    """GG_PART_COLOR_SEP (an extension of partition4, not in the reference):
    the separator part re-ordered by a greedy colouring of its own graph --
    first fit over the separator's nodes in their partition4 order (ascending
    index) -- then by index.  Returns the new pinv, q."""
    nb = node_graph(rp, ci, n)
    pinv, q = np.array(pinv), np.array(q)
    s0 = int(np.sum(np.asarray(node_part) < nparts))
    color = {}
    for i in range(s0, n):
        v = int(q[i])
        used = {color[w] for w in nb[v] if node_part[w] == nparts and w in color}
        c = 0
        while c in used:
            c += 1
        color[v] = c
    seg = sorted(range(s0, n), key=lambda i: (color[int(q[i])], i))
    q[s0:] = [q[i] for i in seg]
    for i in range(s0, n):
        pinv[q[i]] = i
    return pinv, q


def blocks_base(n, nparts):
    """contiguous index ranges (GG_PART_BLOCKS)"""
    return [j * nparts // n for j in range(n)]


def grid_base(rp, ci, n, nparts):
    """GG_PART_GRID (an extension, not in the reference): rectangles of a
    natural-order 2D grid, boxes of a 3D one.  Line length nx = the most
    frequent |offset| > 1 of the pattern (ties: the smallest); plane size nxy =
    the most frequent larger multiple of nx with at least n/8 entries (3D).
    2D: px = the largest divisor of nparts not above sqrt(nparts), py = nparts
    / px, node j = (i, y) -> part (y * py // ny) * px + i * px // nx.  3D: px <=
    py <= pz with pz - px smallest, node (i, y, z) -> part ((z * pz // nz) * py
    + y * py // ny) * px + i * px // nx.  None if not a grid."""
    off = {}
    for r in range(n):
        for k in range(rp[r], rp[r + 1]):
            o = abs(int(ci[k]) - r)
            if 1 < o <= (1 << 24):
                off[o] = off.get(o, 0) + 1
    if not off:
        return None
    nx = min(off, key=lambda o: (-off[o], o))
    if n % nx:
        return None
    planes = [o for o in off if o > nx and o % nx == 0 and off[o] >= n // 8]
    nxy = min(planes, key=lambda o: (-off[o], o)) if planes else None
    if nxy and n % nxy == 0 and n // nxy >= 2:
        ny, nz = nxy // nx, n // nxy
        best = None
        for a in range(1, nparts + 1):
            if nparts % a:
                continue
            for b in range(a, nparts // a + 1):
                if (nparts // a) % b:
                    continue
                c = nparts // a // b
                if c < b:
                    continue
                if best is None or c - a < best[0]:
                    best = (c - a, a, b, c)
        _, px, py, pz = best
    else:
        ny, nz = n // nx, 1
        px = max(d for d in range(1, nparts + 1) if d * d <= nparts and nparts % d == 0)
        py, pz = nparts // px, 1
    if px > nx or py > ny or pz > nz:
        return None
    return [(((j // (nx * ny)) * pz // nz) * py + ((j // nx) % ny) * py // ny) * px + (j % nx) * px // nx
            for j in range(n)]


def permute_dense(A, pinv):
    """P A P^T as a dense array (small test sizes)"""
    D = np.asarray(A.todense())
    n = D.shape[0]
    B = np.zeros_like(D)
    B[np.ix_(pinv, pinv)] = D
    return B


def read_mtx(path):
    """readSparseMatrix: skip '%' lines, 'rows cols nnz', triplets parsed as
    numbers (indices truncated), 1-based -> 0-based, sorted by (row, col)
    (stable here).  Returns (nrows, ncols, rows, cols, vals)."""
    with open(path) as f:
        lines = f.read().splitlines()
    k = 0
    while lines[k].startswith("%"):
        k += 1
    nr, nc, nnz = (int(float(t)) for t in lines[k].split()[:3])
    trip = []
    toks = " ".join(lines[k + 1:]).split()
    for i in range(nnz):
        r, c, v = toks[3 * i:3 * i + 3]
        trip.append((int(float(r)) - 1, int(float(c)) - 1, float(v)))
    trip.sort(key=lambda t: (t[0], t[1]))
    rows = np.array([t[0] for t in trip], np.int64)
    cols = np.array([t[1] for t in trip], np.int64)
    vals = np.array([t[2] for t in trip])
    return nr, nc, rows, cols, vals
