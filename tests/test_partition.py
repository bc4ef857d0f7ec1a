"""Domain decomposition setup and Matrix Market input on the host (no GPU):
gg_host_partition / gg_host_permute / gg_host_block / gg_host_read_mtx against
the restatement in oracle/partition.py (integer work: exact)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import fixture_path
from ggmres import host as H
from ggmres import matrices as M
from oracle import partition as OP

GRIDS = {
    "5pt_40x30": lambda: M.laplacian_5pt(40, 30),
    "7pt_12": lambda: M.grid_7pt(12),
    "powerlaw_800": lambda: M.power_law(800, 6000, seed=9),
    "sherman1": lambda: M.read_rua(fixture_path("sherman1.rua")),
}


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_partition4_blocks_exact(name, nparts):
    """contiguous base partition -> partition4's adjustment, sizes, pinv, q exactly"""
    A = GRIDS[name]()
    n = A.shape[0]
    got = H.partition(A, nparts, H.PART_BLOCKS)
    ref = OP.partition4_adjust(A.indptr, A.indices, n, nparts, OP.blocks_base(n, nparts))
    for k, r in zip(("node_part", "part_size", "pinv", "q"), ref):
        assert np.array_equal(got[k], r), k


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_partition4_color_separator_exact(name, nparts):
    """GG_PART_COLOR_SEP: partition4, then the separator ordered by a greedy
    colouring of its graph; exact vs the restatement, and each colour class of
    the separator is an independent set in A's graph"""
    A = GRIDS[name]()
    n = A.shape[0]
    got = H.partition(A, nparts, H.PART_BLOCKS | H.PART_COLOR_SEP)
    node_part, part_size, pinv, q = OP.partition4_adjust(A.indptr, A.indices, n, nparts,
                                                         OP.blocks_base(n, nparts))
    pinv, q = OP.color_separator(A.indptr, A.indices, n, nparts, node_part, pinv, q)
    assert np.array_equal(got["node_part"], node_part) and np.array_equal(got["part_size"], part_size)
    assert np.array_equal(got["pinv"], pinv) and np.array_equal(got["q"], q)
    # the separator's lower triangle is as deep as the colouring (greedy: at
    # most max degree + 1 classes; well separated 5-point slabs' ladders take 2)
    s0 = n - part_size[nparts]
    nb = OP.node_graph(A.indptr, A.indices, n)
    pos = {int(v): i for i, v in enumerate(q)}
    lev, deg = {}, 0
    for i in range(s0, n):
        v = int(q[i])
        sn = [w for w in nb[v] if node_part[w] == nparts]
        deg = max(deg, len(sn))
        lev[v] = 1 + max([lev[w] for w in sn if pos[w] < i], default=-1)
    if n > s0:
        assert max(lev.values()) + 1 <= deg + 1
        if name == "5pt_40x30" and nparts <= 3:
            assert max(lev.values()) + 1 <= 2


@pytest.mark.parametrize("dims", [(40, 30), (64, 64), (37, 50)])
@pytest.mark.parametrize("nparts", [2, 4, 6, 8])
def test_partition4_grid_blocks_exact(dims, nparts):
    """GG_PART_GRID: px x py rectangles of a 2D grid, then partition4's
    adjustment -- exact vs the restatement; every interior is a full rectangle
    (a row-major sub-grid: the sharded solve's wavefront applies to it) whose
    sides are about nx/px and ny/py"""
    nx, ny = dims
    A = M.laplacian_5pt(nx, ny)
    n = A.shape[0]
    got = H.partition(A, nparts, H.PART_GRID)
    ref = OP.partition4_adjust(A.indptr, A.indices, n, nparts, OP.grid_base(A.indptr, A.indices, n, nparts))
    for k, r in zip(("node_part", "part_size", "pinv", "q"), ref):
        assert np.array_equal(got[k], r), k
    px = max(d for d in range(1, nparts + 1) if d * d <= nparts and nparts % d == 0)
    py = nparts // px
    for p in range(nparts):
        nodes = np.flatnonzero(got["node_part"] == p)
        i, y = nodes % nx, nodes // nx
        w, h = i.max() - i.min() + 1, y.max() - y.min() + 1
        assert w * h == nodes.size                       # a full rectangle
        assert abs(w - nx / px) <= 3 and abs(h - ny / py) <= 3   # two separator layers, rounding
        assert np.all(np.diff(nodes) > 0)                # row-major in the permuted order
        b0 = got["begin"][p]
        assert np.array_equal(got["q"][b0:b0 + nodes.size], nodes)


@pytest.mark.parametrize("dims, nparts, pdims", [((12, 12, 12), 8, (2, 2, 2)), ((16, 10, 12), 4, (1, 2, 2)),
                                                 ((20, 12, 9), 2, (1, 1, 2)), ((10, 12, 14), 6, (1, 2, 3))])
def test_partition4_grid_boxes_3d_exact(dims, nparts, pdims):
    """GG_PART_GRID on a 3D 7-point grid: px x py x pz boxes (the most
    cube-like factorization), exact vs the restatement; every interior a full
    box in row-major order (the tile wavefront applies to it)"""
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz)
    n = A.shape[0]
    got = H.partition(A, nparts, H.PART_GRID)
    ref = OP.partition4_adjust(A.indptr, A.indices, n, nparts, OP.grid_base(A.indptr, A.indices, n, nparts))
    for k, r in zip(("node_part", "part_size", "pinv", "q"), ref):
        assert np.array_equal(got[k], r), k
    px, py, pz = pdims
    for p in range(nparts):
        nodes = np.flatnonzero(got["node_part"] == p)
        i, y, z = nodes % nx, (nodes // nx) % ny, nodes // (nx * ny)
        w, h, d = (v.max() - v.min() + 1 for v in (i, y, z))
        assert w * h * d == nodes.size                    # a full box
        assert abs(w - nx / px) <= 3 and abs(h - ny / py) <= 3 and abs(d - nz / pz) <= 3
        b0 = got["begin"][p]
        assert np.array_equal(got["q"][b0:b0 + nodes.size], nodes)


def test_partition_grid_rejects_non_grid():
    A = M.power_law(800, 6000, seed=9)
    with pytest.raises(Exception):
        H.partition(A, 4, H.PART_GRID)


@pytest.mark.parametrize("name", sorted(GRIDS))
@pytest.mark.parametrize("method", [H.PART_BLOCKS, H.PART_BISECT, H.PART_BLOCKS | H.PART_COLOR_SEP])
@pytest.mark.parametrize("nparts", [2, 4, 8])
def test_arrow_structure(name, method, nparts):
    """interiors are mutually uncoupled; the separator is last; dd_form's blocks
    reassemble the permuted matrix; P A P^T matches the dense permutation"""
    A = GRIDS[name]()
    n = A.shape[0]
    P = H.partition(A, nparts, method)
    pinv, q, begin = P["pinv"], P["q"], P["begin"]
    assert np.array_equal(np.sort(q), np.arange(n)) and np.array_equal(pinv[q], np.arange(n))
    assert P["part_size"].sum() == n
    B = H.permute(A, pinv, q)
    assert np.array_equal(B.toarray(), OP.permute_dense(A, pinv))
    for r in range(n):     # entries of a row sorted by new column
        cols = B.indices[B.indptr[r]:B.indptr[r + 1]]
        assert np.all(np.diff(cols) >= 0)
    for a in range(nparts):
        for b in range(nparts):
            if a != b:
                blk = H.block(B, int(begin[a]), int(begin[a + 1]), int(begin[b]), int(begin[b + 1]))
                assert blk.nnz == 0
    As, E, F, At = H.dd_form(B, begin, nparts)
    s0 = int(begin[nparts])
    R = sp.lil_matrix((n, n))
    for k in range(nparts):
        b0, b1 = int(begin[k]), int(begin[k + 1])
        R[b0:b1, b0:b1] = As[k]
        R[b0:b1, s0:] = E[k]
        R[s0:, b0:b1] = F[k]
    R[s0:, s0:] = At
    assert np.array_equal(R.toarray(), B.toarray())


@pytest.mark.parametrize("nparts", [2, 4, 8])
def test_bisection_balance(nparts):
    """the METIS stand-in splits a grid into parts of equal size (+-1) before
    the separator is taken out, and its separator is a small fraction"""
    A = M.laplacian_5pt(64, 64)
    n = A.shape[0]
    P = H.partition(A, nparts, H.PART_BISECT)
    sizes = P["part_size"][:nparts]
    sep = int(P["part_size"][nparts])
    assert sep < 0.2 * n
    # recover the base sizes: separator nodes belong to some base part; the
    # interiors alone must still be roughly balanced
    assert sizes.min() > 0.5 * sizes.max()


def test_read_mtx_fixtures_exact():
    for f in ("3pt_100.mtx", "5pt_10x10.mtx", "7pt_10x10x10.mtx", "9pt_10x10.mtx"):
        A = H.read_mtx(fixture_path(f))
        nr, nc, rows, cols, vals = OP.read_mtx(fixture_path(f))
        assert A.shape == (nr, nc)
        coo = A.tocoo()
        assert np.array_equal(coo.row, rows) and np.array_equal(coo.col, cols)
        assert np.array_equal(coo.data, vals)
        assert np.array_equal(A.toarray(), M.read_mtx(fixture_path(f)).toarray())


def test_read_mtx_variants(tmp_path):
    p = tmp_path / "s.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n% c\n3 3 4\n1 1 2.5\n2 1 -1\n"
                 "3.0 2.0 -0.5\n3 3 4\n")
    A = H.read_mtx(p)                       # the reference reads every file as general
    assert A.nnz == 4 and A[0, 1] == 0 and A[1, 0] == -1
    S = H.read_mtx(p, expand_symmetric=True)
    assert S.nnz == 6 and S[0, 1] == -1 and S[1, 2] == -0.5
    q = tmp_path / "p.mtx"
    q.write_text("%%MatrixMarket matrix coordinate pattern general\n2 2 2\n2 1\n1 2\n")
    P = H.read_mtx(q)
    assert P.toarray().tolist() == [[0, 1], [1, 0]]
    d = tmp_path / "d.mtx"                  # duplicates kept, in file order
    d.write_text("%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n1 1 2\n2 2 3\n")
    D = H.read_mtx(d)
    assert D.indptr.tolist() == [0, 2, 3] and D.data.tolist() == [1.0, 2.0, 3.0]
    bad = tmp_path / "b.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1\n")
    with pytest.raises(Exception):
        H.read_mtx(bad)
