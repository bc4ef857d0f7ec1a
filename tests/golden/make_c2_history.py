"""Generate the headline configuration's full residual history fixture
(tests/golden/c2_history.npz) from the fp64 oracle restatement (oracle/, test
infrastructure).

    python tests/golden/make_c2_history.py        # ~4 CPU minutes per run, 3 runs in parallel

C2 of BASELINE.json: 1000 x 1000 5-point Laplacian, ILU(0) left
(GMRES_leftILU0, src/gmres.cu:566-717; leftILU src/leftILU.cu:27-336),
GMRES(30), tol 1e-8, b = A*1, x0 = 0, max_iter 20000 -- exactly bench.py's
solve.  Two runs of the same restatement:

  serial  the reference's arithmetic: serial dot/norm sums (src/gmres.cu:45-74)
          and the reference's row division x = acc / d
          (LUSolve_ignoreZero, src/SpMV_compute.cpp:118-133);
  tree    the reference's row arithmetic (x = acc / d) with the device's
          fixed reduction tree (oracle.set_dot_order over the wavefront
          layout): what the GPU's GG_DIV_EXACT mode must reproduce bit for
          bit; against "serial" it isolates the summation order's share of
          the per-entry deviation;
  fma     the device's default arithmetic restated (bench.py's GG_DIV_FMA):
          the device's fixed reduction tree (oracle.set_dot_order over the
          wavefront layout) and the fused rows (oracle.set_div_mode(2, 2)) --
          the GPU must reproduce this one bit for bit; against "tree" it
          isolates the fused rows' share.

Per run: return code, iteration count, inner index, the full residual history
(|s[i+1]|/normb per inner iteration, beta/normb per restart), ||x||_2, sum(x),
and every 997th entry of x (x itself is 8 MB).  Stored with numpy.savez (no
pickles)."""
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "gpu-gmres_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

NX = 1000
RESTART, MAX_ITER, TOL = 30, 20000, 1e-8
X_STRIDE = 997
OUT = os.path.join(HERE, "c2_history.npz")


def run(mode):
    import oracle as O
    from ggmres import matrices as M
    from helpers import device_layout
    A = M.laplacian_5pt(NX)
    b = M.rhs_ones(A)
    L, U = O.ilu0(A)
    if mode in ("tree", "fma"):
        O.set_dot_order(*device_layout(A.shape[0], nx=NX))
    if mode == "fma":
        O.set_div_mode(2, 2)
    try:
        o = O.gmres_left(A, L, U, b, m=RESTART, max_iter=MAX_ITER, tol=TOL)
    finally:
        O.set_dot_order(None)
        O.set_div_mode()
    x = o["x"]
    return mode, {
        "ret_iters_inner": np.array([o["ret"], o["iters"], o["inner"]], np.int64),
        "relres": np.array([o["relres"]]),
        "hist": o["hist"],
        "x_norm_sum": np.array([np.linalg.norm(x), float(np.sum(x))]),
        "x_sample": x[::X_STRIDE].copy(),
    }


def main():
    with Pool(3) as pool:
        res = pool.map(run, ["serial", "tree", "fma"])
    out = {f"{mode}/{k}": v for mode, d in res for k, v in d.items()}
    out["config"] = np.array([NX, RESTART, MAX_ITER, X_STRIDE], np.int64)
    out["tol"] = np.array([TOL])
    np.savez(OUT, **out)
    for mode, d in res:
        print(f"{mode}: ret/iters/inner {d['ret_iters_inner'].tolist()} hist {d['hist'].size} "
              f"relres {d['relres'][0]:.6e}")
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
