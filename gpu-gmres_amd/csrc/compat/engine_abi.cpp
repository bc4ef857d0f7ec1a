// engine_abi.cpp -- the reference's GMRES engine entry points that take the
// Preconditioner plug-in (include/compat/gmres.h; src/gmres.h:356-398,
// src/gmres.cu:2069-2446, 2567-2827), exported with the reference's C++
// signatures and forwarded to the C ABI: the caller's preconditioner object
// becomes a gg_set_precond_user callback (its Dev* methods with device arrays,
// or -- GMRESilu, the host engine -- its Host* methods with host arrays), the
// matrix and vectors are promoted from fp32 to the fp64 engine, x is rounded
// back.  The solver is kept across calls (one setup per matrix; see Ctx).
// Errors print to stderr and return 1 (the reference exits on checkCudaErrors).
#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
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

// The engine state kept across calls (src/gmres.h:82-112: GMRES_GPU_Data exists
// so that a transient caller reuses one workspace across time steps,
// src_thermal/main2.cu:470-506).  One solver per (caller's CSR arrays, n, nnz,
// engine, device; for GMRES_GPU_tran also the caller's GMRES_GPU_Data): the
// first call sets the matrix up (one gg_set_matrix: upload, layout), later
// calls only check that the arrays were not changed in place (an
// order-independent fingerprint of values, row pointers and column indices,
// computed on the device for device arrays) and solve, with b and x promoted
// and x rounded back on the device (gg_solve_device_f32).  A changed matrix
// is set up again.  At most kCacheCap solvers are kept (least recently used
// first out); the reference's engines are not reentrant, neither is this cache
// (one mutex).
struct Ctx {
    gg_solver *s = nullptr;
    int dev = 0, n = 0, nnz = 0, r0 = 0, split = 0;
    bool device = false;
    const void *val = nullptr, *rp = nullptr, *ci = nullptr, *owner = nullptr;
    unsigned long long fp = 0;
    unsigned long long used = 0;
    Plugin pl{nullptr, false, {}, {}};
    ~Ctx()
    {
        if (s) gg_destroy(s);
    }
};
constexpr size_t kCacheCap = 8;
std::mutex g_mu;
// leaked on purpose: a static vector's destructor would run
// gg_destroy (stream sync, hipFree) during static destruction, possibly after
// the HIP runtime has been torn down; the OS reclaims the memory at exit
std::vector<std::unique_ptr<Ctx>> &g_cache = *new std::vector<std::unique_ptr<Ctx>>;
unsigned long long g_tick = 0;

unsigned long long host_fingerprint(const void *p, size_t bytes)
{
    // the device fingerprint's formula (gg_device_fingerprint) on host memory
    const unsigned *w = static_cast<const unsigned *>(p);
    unsigned long long acc = 0;
    for (size_t k = 0; k < bytes / 4; k++) acc += (unsigned long long)w[k] * (unsigned long long)(2 * k + 1);
    return acc;
}

// fingerprint of the caller's CSR (values, row pointers, column indices)
bool csr_fingerprint(bool device, const float *val, const int *rp, const int *ci, int n, int nnz,
                     unsigned long long &fp)
{
    const unsigned long long b[3] = {sizeof(float) * (unsigned long long)nnz,
                                     sizeof(int) * ((unsigned long long)n + 1), sizeof(int) * (unsigned long long)nnz};
    const void *p[3] = {val, rp, ci};
    unsigned long long f[3] = {0, 0, 0};
    if (device) {
        if (gg_device_fingerprint(p, b, 3, f) != GG_OK) return false;
    } else {
        for (int k = 0; k < 3; k++) f[k] = host_fingerprint(p[k], b[k]);
    }
    fp = (f[0] * 0x9E3779B97F4A7C15ull + f[1]) * 0x9E3779B97F4A7C15ull + f[2];
    return true;
}

// the cached solver for this call, set up if missing or stale (nullptr: error reported)
Ctx *context(const char *who, bool device, int split, const float *val, const int *rp, const int *ci, int n,
             const void *owner)
{
    auto fail = [&](const char *what, int rc) -> Ctx * {
        std::fprintf(stderr, "%s: %s: %s (%s)\n", who, what, gg_strerror(rc), gg_last_error());
        return nullptr;
    };
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    Ctx *c = nullptr;
    for (auto &e : g_cache)
        if (e->dev == dev && e->device == device && e->split == split && e->val == val && e->rp == rp &&
            e->ci == ci && e->n == n && e->owner == owner) {
            c = e.get();
            break;
        }
    // a cached entry: one fingerprint round trip over its extent (a changed
    // rp[0] / rp[n] changes the row pointers' fingerprint)
    if (c && c->fp) {
        unsigned long long fp = 0;
        if (!csr_fingerprint(device, val + c->r0, rp, ci + c->r0, n, c->nnz, fp)) return fail("fingerprint", GG_EHIP);
        if (fp == c->fp) {
            c->used = ++g_tick;
            return c;
        }
    }
    int r0 = 0, rn = 0;
    if (!fetch(&r0, rp, sizeof(int), device) || !fetch(&rn, rp + n, sizeof(int), device))
        return fail("row pointers", GG_EHIP);
    const int nnz = rn - r0;
    if (nnz < 0) return fail("row pointers", GG_EINVAL);
    unsigned long long fp = 0;
    if (!csr_fingerprint(device, val + r0, rp, ci + r0, n, nnz, fp)) return fail("fingerprint", GG_EHIP);
    if (!c) {
        if (g_cache.size() >= kCacheCap) {
            auto lru = std::min_element(g_cache.begin(), g_cache.end(),
                                        [](const std::unique_ptr<Ctx> &a, const std::unique_ptr<Ctx> &b) {
                                            return a->used < b->used;
                                        });
            g_cache.erase(lru);
        }
        g_cache.push_back(std::make_unique<Ctx>());
        c = g_cache.back().get();
        c->dev = dev;
        c->device = device;
        c->split = split;
        c->val = val;
        c->rp = rp;
        c->ci = ci;
        c->n = n;
        c->owner = owner;
        int rc = gg_create(dev, &c->s);
        if (rc != GG_OK) {
            g_cache.pop_back();
            return fail("gg_create", rc);
        }
    }
    c->r0 = r0;
    c->nnz = nnz;
    // (re)build: the matrix in fp64 (the reference's float values promoted)
    std::vector<int> hrp(n + 1), hci(nnz);
    std::vector<float> hv(nnz);
    if (!fetch(hrp.data(), rp, sizeof(int) * (n + 1), device) ||
        !fetch(hci.data(), ci + r0, sizeof(int) * nnz, device) || !fetch(hv.data(), val + r0, sizeof(float) * nnz, device))
        return fail("copy in", GG_EHIP);
    for (int &r : hrp) r -= r0;
    std::vector<double> dv(hv.begin(), hv.end());
    c->fp = 0;   // invalid until set up
    int rc = gg_set_matrix(c->s, n, hrp.data(), hci.data(), dv.data());
    if (rc == GG_OK) rc = gg_set_precond_user(c->s, split, call_plugin, &c->pl);
    if (rc != GG_OK) return fail("setup", rc);
    c->fp = fp;
    c->used = ++g_tick;
    return c;
}

// one solve: CSR (fp32 values), b, x (in/out) in device or host memory
int engine(const char *who, bool device, int split, const float *val, const int *rp, const int *ci, int n,
           float *x, const float *b, int m, int max_iter_in, float tol_in, Preconditioner &P, int *iters_out,
           float *tol_out, const void *owner = nullptr)
{
    if (n <= 0 || m < 1) {
        std::fprintf(stderr, "%s: bad sizes n=%d m=%d\n", who, n, m);
        return 1;
    }
    std::lock_guard<std::mutex> lock(g_mu);
    Ctx *c = context(who, device, split, val, rp, ci, n, owner);
    if (!c) return 1;
    c->pl.p = &P;                                // the caller's object of THIS call
    c->pl.host = !device;
    gg_options o{m, max_iter_in, (double)tol_in, 0};
    gg_result res{};
    int rc;
    if (device) {
        rc = gg_solve_device_f32(c->s, b, x, &o, &res);
    } else {
        std::vector<double> dx(x, x + n), db(b, b + n);
        rc = gg_solve(c->s, db.data(), dx.data(), &o, &res);
        if (rc >= 0)
            for (int i = 0; i < n; i++) x[i] = (float)dx[i];
    }
    if (rc < 0) {
        std::fprintf(stderr, "%s: solve: %s (%s)\n", who, gg_strerror(rc), gg_last_error());
        return 1;
    }
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
    if (!Sparse) {
        std::fprintf(stderr, "GMRES_GPU_tran: null argument\n");
        return 1;
    }
    // the solver hangs off the caller's workspace object: one setup per time loop
    return engine("GMRES_GPU_tran", true, 0, Sparse->d_val, Sparse->d_rowIndices, Sparse->d_indices, n, d_x, d_b,
                  m, max_iter, tol, preconditioner, nullptr, nullptr, &gmres_gpu_data);
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
