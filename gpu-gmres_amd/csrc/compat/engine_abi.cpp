// engine_abi.cpp -- the reference's GMRES engine entry points that take the
// Preconditioner plug-in (include/compat/gmres.h; src/gmres.h:356-398,
// src/gmres.cu:2069-2446, 2567-2827), exported with the reference's C++
// signatures and forwarded to the C ABI: the caller's preconditioner object
// becomes a gg_set_precond_user callback (its Dev* methods with device arrays,
// or -- GMRESilu, the host engine -- its Host* methods with host arrays), the
// matrix and vectors are promoted from fp32 to the fp64 engine, x is rounded
// back.  Errors print to stderr and return 1 (the reference exits on
// checkCudaErrors).
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "gmres.h"
#include "ggmres.h"

// the layout is the ABI (x86-64, LP64): src/preconditioner.h:34-84, src/SpMV.h:22-54
// (Preconditioner is polymorphic: offsetof is conditionally supported, exact on
// the Itanium ABI -- vtable pointer first)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Winvalid-offsetof"
static_assert(offsetof(Preconditioner, numRows) == 8 && offsetof(Preconditioner, d_r) == 16 &&
                  offsetof(Preconditioner, d_y) == 40 && offsetof(Preconditioner, s) == 48 &&
                  offsetof(Preconditioner, H) == 72 && offsetof(Preconditioner, d_v) == 80 &&
                  offsetof(Preconditioner, d_ww) == 96 && sizeof(Preconditioner) == 104,
              "Preconditioner layout differs from src/preconditioner.h:34-84");
static_assert(offsetof(SpMatrix, numNZEntries) == 8 && offsetof(SpMatrix, nzentries) == 16 &&
                  sizeof(SpMatrix) == 40 && sizeof(NZEntry) == 12,
              "SpMatrix layout differs from src/SpMV.h:22-42");
static_assert(offsetof(SpMatrixGPU, d_rowIndices) == 16 && sizeof(SpMatrixGPU) == 48,
              "SpMatrixGPU layout differs from src/SpMV.h:44-54");
static_assert(offsetof(GMRES_GPU_Data, s) == 8 && offsetof(GMRES_GPU_Data, d_r) == 40 &&
                  offsetof(GMRES_GPU_Data, d_ww) == 88 && sizeof(GMRES_GPU_Data) == 96,
              "GMRES_GPU_Data layout differs from src/gmres.h:82-112");
#pragma GCC diagnostic pop

namespace {

struct Plugin {
    Preconditioner *p;
    bool host;                   // GMRESilu: Host* methods on host arrays
    std::vector<float> hin, hout;
};

// gg_precond_fn: the engine's fp32 staging arrays (device) -> the plug-in's method
int call_plugin(void *ctx, int op, const float *in, float *out, int n)
{
    Plugin *pl = static_cast<Plugin *>(ctx);
    Preconditioner &P = *pl->p;
    float *i = const_cast<float *>(in);          // the reference's Dev*_ methods take float*
    if (!pl->host) {
        switch (op) {
        case GG_APPLY_MINV: P.DevPrecond(in, out); break;
        case GG_APPLY_LEFT: P.DevPrecond_left(i, out); break;
        case GG_APPLY_RIGHT: P.DevPrecond_right(i, out); break;
        case GG_APPLY_START: P.DevPrecond_starting_value(i, out); break;
        case GG_APPLY_RHS: P.DevPrecond_rhs(i, out); break;
        default: return 1;
        }
        return hipGetLastError() == hipSuccess ? 0 : 1;
    }
    pl->hin.resize(n);
    pl->hout.assign(n, 0.f);
    if (hipMemcpy(pl->hin.data(), in, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    switch (op) {
    case GG_APPLY_MINV: P.HostPrecond(pl->hin.data(), pl->hout.data()); break;
    case GG_APPLY_LEFT: P.HostPrecond_left(pl->hin.data(), pl->hout.data()); break;
    case GG_APPLY_RIGHT: P.HostPrecond_right(pl->hin.data(), pl->hout.data()); break;
    case GG_APPLY_START: P.HostPrecond_starting_value(pl->hin.data(), pl->hout.data()); break;
    case GG_APPLY_RHS: P.HostPrecond_rhs(pl->hin.data(), pl->hout.data()); break;
    default: return 1;
    }
    return hipMemcpy(out, pl->hout.data(), sizeof(float) * n, hipMemcpyHostToDevice) == hipSuccess ? 0 : 1;
}

bool fetch(void *dst, const void *src, size_t bytes, bool device)
{
    if (!bytes) return true;
    if (!device) {
        std::memcpy(dst, src, bytes);
        return true;
    }
    return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess;
}

// one solve: CSR (fp32 values), b, x (in/out) in device or host memory
int engine(const char *who, bool device, int split, const float *val, const int *rp, const int *ci, int n,
           float *x, const float *b, int m, int max_iter_in, float tol_in, Preconditioner &P, int *iters_out,
           float *tol_out)
{
    auto fail = [&](const char *what, int rc) {
        std::fprintf(stderr, "%s: %s: %s (%s)\n", who, what, gg_strerror(rc), gg_last_error());
        return 1;
    };
    if (n <= 0 || m < 1) {
        std::fprintf(stderr, "%s: bad sizes n=%d m=%d\n", who, n, m);
        return 1;
    }
    std::vector<int> hrp(n + 1);
    if (!fetch(hrp.data(), rp, sizeof(int) * (n + 1), device)) return fail("row pointers", GG_EHIP);
    const int nnz = hrp[n] - hrp[0];
    std::vector<int> hci(nnz);
    std::vector<float> hv(nnz), hx(n), hb(n);
    if (!fetch(hci.data(), ci + hrp[0], sizeof(int) * nnz, device) ||
        !fetch(hv.data(), val + hrp[0], sizeof(float) * nnz, device) ||
        !fetch(hx.data(), x, sizeof(float) * n, device) || !fetch(hb.data(), b, sizeof(float) * n, device))
        return fail("copy in", GG_EHIP);
    const int base = hrp[0];
    for (int &r : hrp) r -= base;
    std::vector<double> dv(hv.begin(), hv.end()), dx(hx.begin(), hx.end()), db(hb.begin(), hb.end());
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    gg_solver *s = nullptr;
    int rc = gg_create(dev, &s);
    if (rc != GG_OK) return fail("gg_create", rc);
    Plugin pl{&P, !device, {}, {}};
    gg_result res{};
    rc = gg_set_matrix(s, n, hrp.data(), hci.data(), dv.data());
    if (rc == GG_OK) rc = gg_set_precond_user(s, split, call_plugin, &pl);
    if (rc == GG_OK) {
        gg_options o{m, max_iter_in, (double)tol_in, 0};
        rc = gg_solve(s, db.data(), dx.data(), &o, &res);
    }
    gg_destroy(s);
    if (rc < 0) return fail("solve", rc);
    for (int i = 0; i < n; i++) hx[i] = (float)dx[i];
    if (device ? hipMemcpy(x, hx.data(), sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess
               : (std::memcpy(x, hx.data(), sizeof(float) * n), false))
        return fail("copy out", GG_EHIP);
    if (iters_out) *iters_out = res.iters;
    if (tol_out) *tol_out = (float)res.relres;
    return res.status == GG_OK ? 0 : 1;
}

}  // namespace

// src/gmres.cu:2567-2732 -- left preconditioning by preconditioner.DevPrecond
int GMRES_GPU(SpMatrixGPU *Sparse, SpMatrix *spm, dim3 *grid, dim3 *block, float *d_x, const float *d_b,
              const int n, const int m, int *max_iter, float *tol, Preconditioner &preconditioner)
{
    (void)spm;
    (void)grid;
    (void)block;
    if (!Sparse || !max_iter || !tol) {
        std::fprintf(stderr, "GMRES_GPU: null argument\n");
        return 1;
    }
    return engine("GMRES_GPU", true, 0, Sparse->d_val, Sparse->d_rowIndices, Sparse->d_indices, n, d_x, d_b, m,
                  *max_iter, *tol, preconditioner, max_iter, tol);
}

// src/gmres.cu:2736-2827 -- the same with the limits by value (one time step)
int GMRES_GPU_tran(SpMatrixGPU *Sparse, SpMatrix *spm, dim3 *grid, dim3 *block, float *d_x, const float *d_b,
                   const int n, const int m, const int max_iter, const float tol, Preconditioner &preconditioner,
                   GMRES_GPU_Data &gmres_gpu_data)
{
    (void)spm;
    (void)grid;
    (void)block;
    (void)gmres_gpu_data;
    if (!Sparse) {
        std::fprintf(stderr, "GMRES_GPU_tran: null argument\n");
        return 1;
    }
    return engine("GMRES_GPU_tran", true, 0, Sparse->d_val, Sparse->d_rowIndices, Sparse->d_indices, n, d_x, d_b,
                  m, max_iter, tol, preconditioner, nullptr, nullptr);
}

// src/gmres.cu:2069-2252 -- the split engine on host arrays, Host* methods
int GMRESilu(const float *val, const int *rowIndices, const int *indices, float *x, const float *b,
             const int n, const int m, int *max_iter, float *tol, Preconditioner &preconditioner)
{
    if (!max_iter || !tol) {
        std::fprintf(stderr, "GMRESilu: null argument\n");
        return 1;
    }
    return engine("GMRESilu", false, 1, val, rowIndices, indices, n, x, b, m, *max_iter, *tol, preconditioner,
                  max_iter, tol);
}

// src/gmres.cu:2254-2446 -- the split engine on device arrays, Dev* methods
int GMRESilu_GPU(float *val, int *rowIndices, int *indices, int nnz, float *x, float *b, const int n,
                 const int m, int *max_iter, float *tol, Preconditioner &preconditioner)
{
    (void)nnz;
    if (!max_iter || !tol) {
        std::fprintf(stderr, "GMRESilu_GPU: null argument\n");
        return 1;
    }
    return engine("GMRESilu_GPU", true, 1, val, rowIndices, indices, n, x, b, m, *max_iter, *tol, preconditioner,
                  max_iter, tol);
}
