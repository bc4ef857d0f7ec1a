"""The C-ABI library: builds, loads, exports every declared symbol; host-side
setup code (factorization, grid detection) matches the oracle.  CPU only --
no GPU compute is called here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as O
from conftest import PKG, REPO, fixture_path
from ggmres import matrices as M

HEADERS = ["ggmres.h", "ggmres_host.h", "ggmres_dd.h"]


def declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gg_\w+)\s*\(", txt)))


def exported():
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(PKG, "lib", "libggmres.so")],
                                  text=True)
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_library_exports_every_declared_symbol(ggmres_lib):
    syms = exported()
    for h in HEADERS:
        names = declared(h)
        assert names, h
        missing = [s for s in names if s not in syms]
        assert not missing, f"{h}: not exported: {missing}"
    import ggmres
    assert set(ggmres.EXPORTS) == set(declared("ggmres.h"))
    from ggmres import dd
    assert set(dd.EXPORTS) == set(declared("ggmres_dd.h"))
    for name in ggmres.EXPORTS + dd.EXPORTS:
        getattr(ggmres_lib, name)   # resolvable through ctypes


def test_reference_boundary_classes_exported(ggmres_lib):
    out = subprocess.check_output(
        f"nm -D --defined-only {os.path.join(PKG, 'lib', 'libggmres.so')} | c++filt", shell=True, text=True)
    for sig in ["gmresInterfacePGfloat::setPrecondPG(MySpMatrix*, MySpMatrixDouble*, MySpMatrixDouble*, "
                "MySpMatrix*, MySpMatrix*, MySpMatrix*, MySpMatrix*, MySpMatrix*)",
                "gmresInterfacePGfloat::GMRES_dev_PG()", "gmresInterfacePGfloat::GMRES_host_PG()",
                "gmresInterfacePGfloat::~gmresInterfacePGfloat()",
                "gmresInterfacePG::setPrecondPG(MySpMatrix*, MySpMatrixDouble*, MySpMatrixDouble*, "
                "MySpMatrix*, MySpMatrix*, MySpMatrix*, MySpMatrixDouble*, MySpMatrixDouble*)",
                "gmresInterfacePG::GMRES_host_PG()", "gmresInterfacePG::~gmresInterfacePG()",
                "wrapperGMRESforPG(ucr_cs_dl*, ucr_cs_dl*, ucr_cs_dl*, ucr_cs_dl*, int*, int, gpuETBR*)",
                # the engine ABI with the Preconditioner plug-in (src/gmres.h:356-398)
                "GMRES_GPU(SpMGPU*, SpM*, dim3*, dim3*, float*, float const*, int, int, int*, float*, "
                "Preconditioner&)",
                "GMRES_GPU_tran(SpMGPU*, SpM*, dim3*, dim3*, float*, float const*, int, int, int, float, "
                "Preconditioner&, GMRES_GPU_Data&)",
                "GMRESilu(float const*, int const*, int const*, float*, float const*, int, int, int*, float*, "
                "Preconditioner&)",
                "GMRESilu_GPU(float*, int*, int*, int, float*, float*, int, int, int*, float*, Preconditioner&)"]:
        assert sig in out, sig


@pytest.mark.parametrize("prog, sym", [
    ("pg_driver", "gmresInterfacePGfloat::GMRES_dev_PG()"),
    ("wrapper_driver", "wrapperGMRESforPG(ucr_cs_dl*, ucr_cs_dl*, ucr_cs_dl*, ucr_cs_dl*, int*, int, gpuETBR*)"),
    ("engine_driver", "GMRESilu_GPU(float*, int*, int*, int, float*, float*, int, int, int*, float*, "
                      "Preconditioner&)"),
])
def test_reference_callers_link_unchanged(ggmres_lib, prog, sym):
    """The g++-built stand-ins for the reference's callers (tests/boundary/) take
    their boundary symbols from libggmres.so: undefined in the program, defined
    (same mangled name) in the library, resolved by the dynamic loader."""
    exe = os.path.join(REPO, "tests", "boundary", prog)
    subprocess.check_call(["make", "-s", "-C", os.path.dirname(exe)])
    und = subprocess.check_output(f"nm -u {exe} | c++filt", shell=True, text=True)
    assert sym in und
    ldd = subprocess.check_output(["ldd", exe], text=True)
    lib_line = [ln for ln in ldd.splitlines() if "libggmres.so" in ln]
    assert lib_line and "not found" not in lib_line[0]
    assert os.path.realpath(lib_line[0].split("=>")[1].split("(")[0].strip()) == \
        os.path.realpath(os.path.join(PKG, "lib", "libggmres.so"))


def test_headers_compile_as_c_and_cpp(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "ggmres.h"\n#include "ggmres_host.h"\n#include "ggmres_dd.h"\nint main(void){gg_options o; (void)o; return 0;}\n')
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only",
                           f"-I{REPO}/include", str(c)])
    cc = tmp_path / "t.cpp"
    cc.write_text('#include "gmres_interface_pg.h"\n#include "gpuData.h"\n#include <cstddef>\n'
                  'static_assert(sizeof(gmresInterfacePGfloat) == 120, "layout");\n'
                  'static_assert(offsetof(gmresInterfacePGfloat, rhs_h) == 80, "layout");\n'
                  'static_assert(sizeof(gpuETBR) == 552 && offsetof(gpuETBR, x_single_host) == 184, "layout");\n'
                  'int main(){return 0;}\n')
    subprocess.check_call(["g++", "-std=c++11", "-Wall", "-fsyntax-only",
                           f"-I{REPO}/include/compat", f"-I{REPO}/include", str(cc)])
    ce = tmp_path / "e.cpp"          # the engine ABI header, as a reference caller includes it
    ce.write_text('#include "gmres.h"\n#include <cstddef>\n'
                  'static_assert(sizeof(Preconditioner) == 104, "layout");\n'
                  'static_assert(sizeof(SpMatrixGPU) == 48 && sizeof(SpMatrix) == 40, "layout");\n'
                  'static_assert(sizeof(GMRES_GPU_Data) == 96, "layout");\n'
                  'int main(){return 0;}\n')
    subprocess.check_call(["g++", "-std=c++11", "-Wall", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", f"-I{REPO}/include/compat", f"-I{REPO}/include", str(ce)])


def test_status_strings_and_version(ggmres_lib):
    ggmres_lib.gg_strerror.restype = ctypes.c_char_p
    assert ggmres_lib.gg_abi_version() == 1
    assert ggmres_lib.gg_strerror(0) == b"converged"
    assert ggmres_lib.gg_strerror(1) == b"not converged"
    assert ggmres_lib.gg_strerror(-3) == b"zero pivot in factorization"


# ------------------------------------------------------ host setup vs oracle
PI = ctypes.POINTER(ctypes.c_int)
PD = ctypes.POINTER(ctypes.c_double)


def host_factor(lib, A, level=None):
    A = O.csr(A)
    n = A.n
    lrp = np.zeros(n + 1, np.int32)
    urp = np.zeros(n + 1, np.int32)
    lci, lv, uci, uv = PI(), PD(), PI(), PD()
    args = [ctypes.c_int(n), A.rp.ctypes.data_as(PI), A.ci.ctypes.data_as(PI), A.v.ctypes.data_as(PD),
            lrp.ctypes.data_as(PI), ctypes.byref(lci), ctypes.byref(lv),
            urp.ctypes.data_as(PI), ctypes.byref(uci), ctypes.byref(uv)]
    rc = lib.gg_host_ilu0(*args) if level is None else lib.gg_host_iluk(ctypes.c_int(level), *args)
    if rc != 0:
        return rc, None, None

    def take(rp, ci, v):
        nnz = int(rp[n])
        out = O.CSR(n, rp, np.ctypeslib.as_array(ci, (max(nnz, 1),))[:nnz].copy(),
                    np.ctypeslib.as_array(v, (max(nnz, 1),))[:nnz].copy())
        lib.gg_host_free(ctypes.cast(ci, ctypes.c_void_p))
        lib.gg_host_free(ctypes.cast(v, ctypes.c_void_p))
        return out
    return 0, take(lrp, lci, lv), take(urp, uci, uv)


CASES = ["5pt_10x10.mtx", "7pt_10x10x10.mtx", "9pt_10x10.mtx", "3pt_100.mtx", "sherman1.rua"]


def load(name):
    return M.read_rua(fixture_path(name)) if name.endswith(".rua") else M.read_mtx(fixture_path(name))


@pytest.mark.parametrize("name", CASES)
def test_host_ilu0_bitexact_vs_oracle(ggmres_lib, name):
    A = load(name)
    rc, L, U = host_factor(ggmres_lib, A)
    assert rc == 0
    Lo, Uo = O.ilu0(A)
    for a, b in ((L, Lo), (U, Uo)):
        assert np.array_equal(a.rp, b.rp) and np.array_equal(a.ci, b.ci)
        assert np.array_equal(a.v, b.v)   # bit-exact


def test_host_ilu0_c1_bitexact(ggmres_lib):
    A = M.laplacian_5pt(100)
    rc, L, U = host_factor(ggmres_lib, A)
    Lo, Uo = O.ilu0(A)
    assert rc == 0 and np.array_equal(L.v, Lo.v) and np.array_equal(U.v, Uo.v)


@pytest.mark.parametrize("name,k", [("5pt_10x10.mtx", 1), ("7pt_10x10x10.mtx", 1), ("9pt_10x10.mtx", 2),
                                    ("sherman1.rua", 1)])
def test_host_iluk_bitexact_vs_oracle(ggmres_lib, name, k):
    A = load(name)
    rc, L, U = host_factor(ggmres_lib, A, level=k)
    try:
        Lo, Uo = O.iluk(A, k)
    except ZeroDivisionError:
        assert rc == -3
        return
    assert rc == 0
    for a, b in ((L, Lo), (U, Uo)):
        assert np.array_equal(a.rp, b.rp) and np.array_equal(a.ci, b.ci)
        assert np.array_equal(a.v, b.v)


def host_iluk_pattern(lib, A, level, threads):
    A = O.csr(A)
    prow = np.zeros(A.n + 1, np.int32)
    pcol = PI()
    rc = lib.gg_host_iluk_pattern(ctypes.c_int(level), ctypes.c_int(A.n), A.rp.ctypes.data_as(PI),
                                  A.ci.ctypes.data_as(PI), ctypes.c_int(threads),
                                  prow.ctypes.data_as(PI), ctypes.byref(pcol))
    assert rc == 0
    nnz = int(prow[-1])
    cols = np.ctypeslib.as_array(pcol, (max(nnz, 1),))[:nnz].copy()
    lib.gg_host_free(ctypes.cast(pcol, ctypes.c_void_p))
    return prow, cols


def random_nonsym(n, per_row, seed):
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(n), per_row)
    cols = rng.integers(0, n, n * per_row)
    A = sp.csr_matrix((rng.standard_normal(n * per_row), (rows, cols)), shape=(n, n))
    A = A + sp.diags(np.abs(A).sum(axis=1).A1 + 1.0)
    A.sum_duplicates()
    A.sort_indices()
    return A.tocsr()


@pytest.mark.parametrize("case", CASES + ["rand300", "rand1000"])
def test_host_iluk_pattern_row_parallel(ggmres_lib, case):
    """The row-parallel symbolic phase (level 1 by L x U, level >= 2 by
    incomplete fill paths) equals lofC's pattern (src/iluk.cpp:193-334) row by
    row, for any thread count."""
    A = (random_nonsym(300, 4, 11) if case == "rand300" else
         random_nonsym(1000, 3, 12) if case == "rand1000" else load(case))
    for k in (0, 1, 2, 3, 4):
        try:
            Lo, Uo = O.iluk(A, k)
        except ZeroDivisionError:
            continue
        ref_rp = np.zeros(Lo.n + 1, np.int64)
        ref_ci = []
        for r in range(Lo.n):
            row = np.union1d(Lo.ci[Lo.rp[r]:Lo.rp[r + 1]], Uo.ci[Uo.rp[r]:Uo.rp[r + 1]])
            ref_ci.append(row)
            ref_rp[r + 1] = ref_rp[r] + row.size
        ref_ci = np.concatenate(ref_ci)
        for threads in (1, 4):
            prow, cols = host_iluk_pattern(ggmres_lib, A, k, threads)
            assert np.array_equal(prow, ref_rp), (case, k, threads)
            assert np.array_equal(cols, ref_ci), (case, k, threads)


def test_host_iluk_zero_pivot(ggmres_lib):
    import scipy.sparse as sp
    A = sp.csr_matrix(np.array([[0.0, 1.0], [1.0, 1.0]]))
    rc, _, _ = host_factor(ggmres_lib, A, level=1)
    assert rc == -3


def wave(lib, L, U):
    nx, ny = ctypes.c_int(), ctypes.c_int()
    ok = lib.gg_host_wave2d(ctypes.c_int(L.n), L.rp.ctypes.data_as(PI), L.ci.ctypes.data_as(PI),
                            L.v.ctypes.data_as(PD), U.rp.ctypes.data_as(PI), U.ci.ctypes.data_as(PI),
                            U.v.ctypes.data_as(PD), ctypes.byref(nx), ctypes.byref(ny))
    return ok, nx.value, ny.value


def test_wavefront_detection(ggmres_lib):
    for nx, ny in ((100, 100), (37, 64), (200, 3)):
        A = M.laplacian_5pt(nx, ny)
        L, U = O.ilu0(A)
        assert wave(ggmres_lib, L, U) == (1, nx, ny)
    # 3D 7-pt and 9-pt factors do not have the 2D 5-pt structure
    for A in (M.grid_7pt(8), load("9pt_10x10.mtx")):
        L, U = O.ilu0(A)
        assert wave(ggmres_lib, L, U)[0] == 0
    # ILU(1) / ILU(2) factors of a 5-point grid: the skewed wavefront (fill at
    # offsets nx-1, nx-2); ILU(3) adds offset nx-3: beyond the kernel's skew 3
    for k in (1, 2):
        L, U = O.iluk(M.laplacian_5pt(30), k)
        assert wave(ggmres_lib, L, U) == (1, 30, 30)
    L, U = O.iluk(M.laplacian_5pt(30), 3)
    assert wave(ggmres_lib, L, U)[0] == 0


def layout(lib, L, U):
    n = L.n
    slot = np.zeros(max(n, 1), np.int64)
    info = np.zeros(9, np.int32)
    ok = lib.gg_host_wave_layout(ctypes.c_int(n), L.rp.ctypes.data_as(PI), L.ci.ctypes.data_as(PI),
                                 L.v.ctypes.data_as(PD), U.rp.ctypes.data_as(PI), U.ci.ctypes.data_as(PI),
                                 U.v.ctypes.data_as(PD), slot.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                                 info.ctypes.data_as(PI))
    return ok, slot[:n], info


@pytest.mark.parametrize("dims", [(20, 30, 7), (16, 70, 5), (8, 8, 300), (130, 3, 4), (100, 100, 1), (37, 64, 1)])
def test_wave_layout_matches_restatement(ggmres_lib, dims):
    """The solver's wavefront vector layout (gg_host_wave_layout: 2D bands, 3D
    8-line x 8-plane tiles) equals the restatement the order-matched oracle
    uses (tests/helpers.py device_layout), and is one-to-one."""
    from helpers import device_layout
    nx, ny, nz = dims
    A = M.grid_7pt(nx, ny, nz, upwind=0.1) if nz > 1 else M.laplacian_5pt(nx, ny)
    n = A.shape[0]
    L, U = O.ilu0(A)
    ok, slot, info = layout(ggmres_lib, L, U)
    assert ok == 1
    assert info[0] == (3 if nz > 1 else 2) and tuple(info[1:4]) == (nx, ny, nz)
    if nz > 1:
        assert info[6] == (ny + 7) // 8 and info[7] == (nz + 7) // 8 and info[4] == info[6] * info[7]
        assert info[5] == (nx + 14 + 15) // 16 * 16
    assert len(np.unique(slot)) == n
    lay2nat, _ = device_layout(n, nx, ny if nz > 1 else None)
    assert np.array_equal(lay2nat[slot], np.arange(n))


def split_layout(lib, L, U):
    n = L.n
    slot = np.zeros(max(n, 1), np.int64)
    info = np.zeros(9, np.int32)
    ok = lib.gg_host_split_layout(ctypes.c_int(n), L.rp.ctypes.data_as(PI), L.ci.ctypes.data_as(PI),
                                  L.v.ctypes.data_as(PD), U.rp.ctypes.data_as(PI), U.ci.ctypes.data_as(PI),
                                  U.v.ctypes.data_as(PD), slot.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                                  info.ctypes.data_as(PI))
    return ok, slot[:n], info


@pytest.mark.parametrize("grid, stride", [(60, 20), (150, 50), (64, 30)])
def test_split_layout_bordered_netlist(ggmres_lib, tmp_path, grid, stride):
    """An MNA power grid pivoted with its pads and branch rows first
    (mna_pivot_order) is a bordered grid for the split engine: the tail of
    2 x pads rows at slots [0, tail), the mesh as a 2D wavefront after them --
    the layout the order-matched oracle restates (device_layout border=)."""
    from helpers import device_layout, make_split, netlist_system
    A, prow, pcol, nt = netlist_system(str(tmp_path / "pg.sp"), grid, stride)
    n = A.shape[0]
    P = make_split(A, seed=3, perm=(prow, pcol))
    ok, slot, info = split_layout(ggmres_lib, P.L, P.U)
    assert ok == 1 and info[0] == 5 and tuple(info[1:3]) == (grid, grid)
    assert info[6] == nt and info[7] == (nt + 63) // 64 * 64
    assert len(np.unique(slot)) == n
    lay2nat, _ = device_layout(n, grid, border=nt)
    assert np.array_equal(lay2nat[slot], np.arange(n))


def test_split_layout_plain_and_rcm(ggmres_lib, monkeypatch):
    """grid-shaped split factors: the plain 2D layout; a random symmetric
    permutation of the grid: the flow path's RCM layout -- a permutation whose
    bandwidth is back near the grid's line length -- or, with GG_FLOW_RCM=0,
    natural order"""
    from helpers import make_split
    A = M.laplacian_5pt(48, 40)
    P = make_split(A, seed=9, identity_perm=True)
    ok, slot, info = split_layout(ggmres_lib, P.L, P.U)
    assert ok == 1 and info[0] == 2 and info[6] == 0 and tuple(info[1:3]) == (48, 40)
    P = make_split(A, seed=9)
    ok, slot, info = split_layout(ggmres_lib, P.L, P.U)
    n = A.shape[0]
    assert ok == 1 and info[0] == 6 and np.array_equal(np.sort(slot), np.arange(n))
    # bandwidth of L + U in the relabeled order vs in the random order
    rows = np.repeat(np.arange(n), np.diff(P.L.rp))
    bw_rand = np.max(np.abs(rows - P.L.ci))
    bw_rcm = np.max(np.abs(slot[rows] - slot[P.L.ci]))
    assert bw_rcm <= 3 * 48 < bw_rand
    monkeypatch.setenv("GG_FLOW_RCM", "0")
    assert split_layout(ggmres_lib, P.L, P.U)[0] == 0
