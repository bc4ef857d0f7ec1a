// gmres_host.h -- the host GMRESilu engine (gmres_host.cpp) behind the PG
// classes' GMRES_host_PG (csrc/compat/interface_pg.cpp).
#pragma once

#include <vector>

namespace gg {

// A (CSR) and the ILU++ split preconditioner of MyILUPP (src/preconditioner.h):
// L with its diagonal last in each row, U with its diagonal first, the middle
// diagonal, the row / column permutations and the two scalings, all fp64
struct HostSplitEngine {
    int n = 0;
    std::vector<int> arp, aci, lrp, lci, urp, uci, prow, pcol;
    std::vector<double> av, lv, uv, mid, ls, rs;
};

// GMRESilu (src/gmres.cu:2069-2252) in fp64: x in = initial guess, out =
// solution; *max_iter / *tol in = limits, out = iterations / relative residual
// as the reference writes them; returns 0 converged, 1 not
int gmres_split_host(const HostSplitEngine &E, const double *b, double *x, int m, int *max_iter, double *tol,
                     int *inner_iters);
int host_threads();   // threads of the element-wise loops (GG_HOST_THREADS, <= 16)

}  // namespace gg
