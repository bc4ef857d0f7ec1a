"""Device vs host ILU(0) / ILU(k) factorization time (GPU).
python tools/ilu_bench.py [grid ...]  -> per grid: device ms (k_ilu0_columns +
gathers, hipEvents), host ms (ilu0_left through gg_host_ilu0); ILU(1) and
ILU(2): device ms (k_iluk_rows + gather) vs host ms (gg_host_iluk), equal?"""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "gpu-gmres_amd"))
import numpy as np                      # noqa: E402
import ggmres as G                      # noqa: E402
from ggmres import matrices as M        # noqa: E402

lib = G.lib()
PI, PD = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)
s = G.Solver()
for grid in [int(a) for a in sys.argv[1:]] or [300, 1000]:
    A = M.laplacian_5pt(grid)
    n = A.shape[0]
    s.set_matrix(A)
    s.ilu0_device_values()                          # warm-up (code load)
    fv, ms = s.ilu0_device_values()
    lrp, urp = np.zeros(n + 1, np.int32), np.zeros(n + 1, np.int32)
    lci, lv, uci, uv = PI(), PD(), PI(), PD()
    t = time.perf_counter()
    rc = lib.gg_host_ilu0(ctypes.c_int(n), A.indptr.ctypes.data_as(PI), A.indices.ctypes.data_as(PI),
                          A.data.ctypes.data_as(PD), lrp.ctypes.data_as(PI), ctypes.byref(lci),
                          ctypes.byref(lv), urp.ctypes.data_as(PI), ctypes.byref(uci), ctypes.byref(uv))
    host_ms = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    s.set_precond_ilu0_device()
    dev_setup_ms = (time.perf_counter() - t) * 1e3
    t = time.perf_counter()
    s.set_precond_ilu0()
    host_setup_ms = (time.perf_counter() - t) * 1e3
    print(f"grid {grid}: n={n} device factor {ms:.2f} ms, host ilu0_left {host_ms:.1f} ms (rc {rc}); "
          f"set_precond_ilu0_device {dev_setup_ms:.1f} ms vs set_precond_ilu0 {host_setup_ms:.1f} ms")
    for k in (1, 2):
        s.iluk_device_factors(k)                    # warm-up
        (dl, du, dms) = s.iluk_device_factors(k)
        lci, lv, uci, uv = PI(), PD(), PI(), PD()
        t = time.perf_counter()
        rc = lib.gg_host_iluk(ctypes.c_int(k), ctypes.c_int(n), A.indptr.ctypes.data_as(PI),
                              A.indices.ctypes.data_as(PI), A.data.ctypes.data_as(PD),
                              lrp.ctypes.data_as(PI), ctypes.byref(lci), ctypes.byref(lv),
                              urp.ctypes.data_as(PI), ctypes.byref(uci), ctypes.byref(uv))
        host_ms = (time.perf_counter() - t) * 1e3
        nl, nu = int(lrp[n]), int(urp[n])
        same = (np.array_equal(dl[0], lrp) and np.array_equal(du[0], urp) and
                np.array_equal(dl[2], np.ctypeslib.as_array(lv, shape=(nl,))) and
                np.array_equal(du[2], np.ctypeslib.as_array(uv, shape=(nu,))))
        print(f"grid {grid}: ILU({k}) nnz(L)+nnz(U) = {nl + nu}: device numeric {dms:.2f} ms, "
              f"host lofC+ilukC {host_ms:.1f} ms (rc {rc}), factors identical: {same}")
s.close()
