"""SPICE power-grid netlist -> MNA (gg_host_read_netlist, csrc/host/netlist.cpp)
against the oracle's restatement of parser() + stampG/stampC/stampB
(oracle/netlist.py; src/parser.cpp:69-272, 1904-2886): bit-exact G, C, B,
source waveforms, node numbering, ports; and (GPU) a netlist driven through
the device transient driver.  Parity unpinned against the reference itself (it
ships no netlists; its parser is not buildable here)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from oracle import netlist as ON            # noqa: E402
from ggmres import host as H                # noqa: E402


def grid_netlist(path, nx, ny, seed=0, extras=True, include=True):
    """An ibmpg-like grid: C to ground first (rows = row-major node order),
    R between neighbours, current sources (DC / PWL with '+' lines / PULSE);
    extras: a pad voltage source behind a resistor, an inductor, a cap between
    two nodes, 'gnd', lowercase letters, duplicate stamps, SPICE suffixes."""
    rng = np.random.default_rng(seed)
    nm = lambda j, i: f"n1_{j}_{i}"
    L = ["* synthetic power grid", ".tran 10p 2n"]
    for j in range(ny):
        for i in range(nx):
            L.append(f"C{j}_{i} {nm(j, i)} {'gnd' if (i + j) % 7 == 0 else '0'} {rng.integers(1, 90)}f")
    R = []
    for j in range(ny):
        for i in range(nx):
            if i + 1 < nx:
                R.append(f"R{j}_{i}h {nm(j, i)} {nm(j, i + 1)} {rng.uniform(0.1, 2.0):.4f}")
            if j + 1 < ny:
                R.append(f"r{j}_{i}v {nm(j, i)} {nm(j + 1, i)} {rng.integers(1, 900)}m")
    if include:
        inc = path + ".inc"
        with open(inc, "w") as f:
            f.write("\n".join(R[len(R) // 2:]) + "\n")
        L += R[:len(R) // 2] + [f'.include "{os.path.basename(inc)}"']
    else:
        L += R
    L.append(f"R_dup {nm(0, 0)} {nm(0, 1)} 1.5k")               # duplicate stamp
    L.append(f"I1 {nm(1, 1)} 0 {1e-3:g}")
    L.append(f"I2 {nm(2, 3)} 0 PWL(0.5n 1m 1n 2m)")
    L.append("+ 1.5n 0.5m")
    L.append("+ 2n 3m")
    L.append(f"i3 {nm(ny - 1, nx - 1)} 0 0 PULSE(0, 10m, 0.2n, 0.1n, 0.1n, 0.5n, 1n)")
    L.append(f"I4 0 {nm(ny // 2, nx // 2)} PWL(0 0 1n 4m)")
    if extras:
        L.append(f"Rpad {nm(0, 0)} _X_{nm(0, 0)} 10m")
        L.append(f"V1 _X_{nm(0, 0)} 0 1.8")
        L.append(f"L1 {nm(0, nx - 1)} {nm(1, nx - 1)} 1n")
        L.append(f"Cc {nm(2, 2)} {nm(2, 3)} 5f")
        L.append(f"V2 {nm(3, 0)} gnd PWL(0 1.8 1n 1.7)")
        L.append(f"V3 {nm(3, 1)} 0 0 PULSE(1.8, 1.7, 1n, 0.1n, 0.1n, 1n, 3n)")
    L.append(f".print tran v({nm(0, 0)}) v({nm(ny - 1, nx - 1)}) v(nope)")
    L.append(".end")
    with open(path, "w") as f:
        f.write("\n".join(L) + "\n")
    return path


def as_dict(M):
    M = M.tocoo()
    return {(int(i), int(j)): float(v) for i, j, v in zip(M.row, M.col, M.data)}


@pytest.mark.parametrize("dims,extras,include", [((6, 5), True, True), ((9, 9), False, False),
                                                 ((30, 17), True, True)])
def test_netlist_matches_oracle(tmp_path, dims, extras, include):
    p = grid_netlist(str(tmp_path / "pg.sp"), *dims, seed=dims[0], extras=extras, include=include)
    nl = H.Netlist(p)
    o = ON.read_netlist(p)
    for k in ("n", "n_nodes", "n_l", "n_v", "n_i", "tstep", "tstop"):
        assert getattr(nl, k) == o[k], k
    for name in ("G", "C", "B"):
        d = as_dict(getattr(nl, name))
        od = o[name]
        assert d.keys() == od.keys(), name
        for key in od:                                      # bit-exact sums in netlist order
            assert np.float64(d[key]).tobytes() == np.float64(od[key]).tobytes(), (name, key)
    assert len(nl.sources) == len(o["sources"])
    for (k, par), (ok, opar) in zip(nl.sources, o["sources"]):
        assert k == ok and np.array_equal(par, np.array(opar, np.float64))
    assert list(nl.ports) == o["ports"]
    assert nl.ports[-1] == -1


def test_netlist_semantics(tmp_path):
    """Spot checks of the restated rules on a hand-written netlist."""
    p = str(tmp_path / "small.sp")
    with open(p, "w") as f:
        f.write("* tiny\n.tran 1p 1n\nR1 a b 2k\nR2 b 0 1meg\nC1 a 0 3p\nL1 b c 4n\n"
                "V1 c 0 1.5\nI1 a b 2m\nI2 b 0 PWL(1n 5m 2n 6m)\n.print tran v(b)\n.end\n")
    nl = H.Netlist(p)
    assert (nl.n_nodes, nl.n_l, nl.n_v, nl.n_i, nl.n) == (3, 1, 1, 2, 5)
    G = nl.G.toarray()
    assert G[0, 0] == 1 / 2e3 and G[0, 1] == -1 / 2e3
    assert G[1, 1] == 1 / 2e3 + 1 / 1e6                     # 'meg' = 1e6 (StrToNum)
    assert G[3, 1] == -1 and G[1, 3] == 1 and G[3, 2] == 1 and G[2, 3] == -1    # L branch row 3
    assert G[2, 4] == 1 and G[4, 2] == -1                   # V branch row 4
    C = nl.C.toarray()
    assert C[0, 0] == 3e-12 and C[3, 3] == 4e-9
    B = nl.B.toarray()
    assert B[4, 0] == -1 and B[0, 1] == -1 and B[1, 1] == 1 and B[1, 2] == -1
    assert nl.sources[0][0] == 0 and np.array_equal(nl.sources[0][1], [1.5])       # V1: DC
    assert nl.sources[1][0] == 0 and np.array_equal(nl.sources[1][1], [2e-3])      # I1: DC
    k, par = nl.sources[2]
    assert k == 2 and np.array_equal(par, [0.0, 5e-3, 1e-9, 5e-3, 2e-9, 6e-3])  # (0, v0) prepended
    assert list(nl.ports) == [1]


def test_netlist_missing_file(tmp_path):
    from ggmres import GGError
    with pytest.raises(GGError):
        H.Netlist(str(tmp_path / "none.sp"))


@pytest.mark.parametrize("bad", ["L1 b c", "V1 c 0", "I1 a", "R1 a b", "C1 a"])
def test_netlist_short_element_line_rejected(tmp_path, bad):
    """An element line without two nodes and a value is rejected, naming the
    line, in both passes alike (no reserved branch row left unstamped)."""
    from ggmres import GGError
    p = str(tmp_path / "short.sp")
    with open(p, "w") as f:
        f.write(f"* x\nR0 a b 1k\nL0 b 0 1n\n{bad}\nV0 a 0 1\n.end\n")
    with pytest.raises(GGError) as ei:
        H.Netlist(p)
    assert bad in str(ei.value)
    with pytest.raises(ValueError):
        ON.read_netlist(p)


@pytest.mark.parametrize("spelling", ["PULSE(0, 10m, 0.2n, 0.1n, 0.1n, 0.5n, 1n)",
                                      "PULSE (0, 10m, 0.2n, 0.1n, 0.1n, 0.5n, 1n)",
                                      "pulse( 0 10m 0.2n 0.1n 0.1n 0.5n 1n )",
                                      "PULSE(0,10m,0.2n,0.1n,0.1n,0.5n,1n)"])
def test_netlist_pulse_spellings(tmp_path, spelling):
    """PULSE arguments are read between the parentheses, blank- or
    comma-separated: every spelling gives the reference spelling's values."""
    p = str(tmp_path / "pulse.sp")
    with open(p, "w") as f:
        f.write(f"* x\nR0 a 0 1k\nC0 a 0 1p\nI1 a 0 0 {spelling}\n.end\n")
    nl = H.Netlist(p)
    o = ON.read_netlist(p)
    want = [0.0, 10e-3, 0.2e-9, 0.1e-9, 0.1e-9, 0.5e-9, 1e-9]
    k, par = nl.sources[0]
    assert k == 1 and np.allclose(par, want, rtol=0, atol=1e-25)
    assert o["sources"][0][0] == 1 and np.array_equal(np.array(o["sources"][0][1]), par)
    ref = H.Netlist(_write(tmp_path / "ref.sp", "* x\nR0 a 0 1k\nC0 a 0 1p\n"
                           "I1 a 0 0 PULSE(0, 10m, 0.2n, 0.1n, 0.1n, 0.5n, 1n)\n.end\n"))
    assert np.array_equal(ref.sources[0][1], par)


def test_netlist_pulse_malformed_is_dc_zero(tmp_path):
    p = _write(tmp_path / "m.sp", "* x\nR0 a 0 1k\nI1 a 0 0 PULSE(1, 2, 3)\n.end\n")
    nl = H.Netlist(p)
    assert nl.sources[0][0] == 0 and np.array_equal(nl.sources[0][1], [0.0])
    assert ON.read_netlist(p)["sources"][0] == (0, [0.0])


def _write(path, text):
    with open(str(path), "w") as f:
        f.write(text)
    return str(path)


@pytest.mark.gpu
def test_netlist_transient_on_device(tmp_path):
    """RC grid netlist (C to ground, R mesh, current sources) -> A = G + C/h,
    transient_src on the device vs the restated step driver (serial order)."""
    import ggmres
    import oracle as O
    nx, ny = 48, 40
    p = grid_netlist(str(tmp_path / "rc.sp"), nx, ny, seed=3, extras=False, include=False)
    nl = H.Netlist(p)
    h = 1e-11
    A, cdiag, nodes, kinds, ptr, data = nl.transient_inputs(h)
    srcs = [(int(kinds[k]), data[ptr[k]:ptr[k + 1]]) for k in range(len(kinds))]
    ports = nl.ports[nl.ports >= 0]
    n = A.shape[0]
    x0 = np.zeros(n)
    L, U = O.ilu0(A)
    o = O.transient(A, L, U, 20, h, cdiag, nodes, None, ports, x0, m=32, max_iter=10000, tol=1e-9,
                    sources=srcs)
    s = ggmres.Solver(0)
    try:
        s.set_matrix(A)
        s.set_precond_ilu0()
        assert s.uses_wavefront                  # C lines first: natural row-major grid order
        g = s.transient_src(20, h, cdiag, nodes, srcs, ports, x0, restart=32, max_iter=10000, tol=1e-9)
    finally:
        s.close()
    assert g["iters_total"] == o["iters_total"]
    scale = np.max(np.abs(o["ports"]))
    assert scale > 0
    assert np.max(np.abs(g["ports"] - o["ports"])) <= 1e-10 * scale
    assert np.linalg.norm(g["x"] - o["x"]) <= 1e-10 * np.linalg.norm(o["x"])
