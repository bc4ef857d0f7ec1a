// engine_driver.cpp -- a caller of the reference's engine entry points with the
// Preconditioner plug-in (src/gmres.h:356-398, src/preconditioner.h:34-84),
// compiled with g++ and linked against libggmres.so: it derives its own
// preconditioner from Preconditioner -- Jacobi, M = D (left: DevPrecond /
// HostPrecond = D^-1; split: Ml = Mr = D^-1/2, start = D^1/2, as an ILU++-style
// object would expose them) -- in the way src_thermal/main1.cu:335-397 builds
// one and hands it to GMRES_GPU.  Its Dev* methods move the fp32 vectors through
// host memory (g++ has no kernels); it counts its calls.
//
//   engine_driver IN OUT
// IN  (little-endian int32 unless noted): mode (0 GMRES_GPU, 1 GMRES_GPU_tran,
//     2 GMRESilu_GPU, 3 GMRESilu), n, nnz, m, max_iter, float tol;
//     rp[n+1] ci[nnz] float val[nnz] float b[n] float x0[n]
// OUT int32 return code, int32 max_iter (out), float tol (out), int32 calls[5]
//     (DevPrecond/HostPrecond, _left, _right, _starting_value, _rhs), float x[n]
// mode 4 (a transient caller, src_thermal/main2.cu:470-506): kSteps time steps
//     of GMRES_GPU_tran with ONE GMRES_GPU_Data, b_t = b (1 + t/100), x warm-
//     started; then the same steps through the C ABI directly (one gg_solver set
//     up once, gg_solve_device_f32, the same plug-in as a gg_precond_fn).
//     OUT int32 rc (last step), int32 gg_set_matrix calls during the
//     GMRES_GPU_tran loop, double ms per step (GMRES_GPU_tran), double ms per
//     step (C ABI), float x[n] (GMRES_GPU_tran's last step), float x[n] (C ABI)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "ggmres.h"
#include "gmres.h"

namespace {

FILE *g_in;

template <class T>
std::vector<T> rd(size_t count)
{
    std::vector<T> v(count);
    if (count && std::fread(v.data(), sizeof(T), count, g_in) != count) {
        std::fprintf(stderr, "engine_driver: short input\n");
        std::exit(2);
    }
    return v;
}

void check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        std::fprintf(stderr, "engine_driver: %s: %s\n", what, hipGetErrorString(e));
        std::exit(3);
    }
}

class Jacobi : public Preconditioner {
public:
    std::vector<float> d;     // the diagonal of A
    int calls[5] = {0, 0, 0, 0, 0};

    void Initilize(const MySpMatrix &A) override
    {
        numRows = A.numRows;
        d.assign(numRows, 1.0f);
        for (int r = 0; r < numRows; r++)
            for (int k = A.rowIndices[r]; k < A.rowIndices[r + 1]; k++)
                if (A.indices[k] == r) d[r] = A.val[k];
        d_r = d_rr = d_bb = d_y = s = cs = sn = H = d_v = d_w = d_ww = nullptr;
    }
    // host kernels of the operators: 0 = D^-1, 1 = D^-1/2, 2 = D^1/2
    void host_op(int kind, const float *in, float *out) const
    {
        for (int i = 0; i < numRows; i++)
            out[i] = kind == 0 ? in[i] / d[i] : kind == 1 ? in[i] / std::sqrt(d[i]) : in[i] * std::sqrt(d[i]);
    }
    void dev_op(int kind, const float *in, float *out) const
    {
        std::vector<float> h(numRows), o(numRows);
        check(hipMemcpy(h.data(), in, sizeof(float) * numRows, hipMemcpyDeviceToHost), "D2H");
        host_op(kind, h.data(), o.data());
        check(hipMemcpy(out, o.data(), sizeof(float) * numRows, hipMemcpyHostToDevice), "H2D");
    }
    void HostPrecond(const ValueType *i, ValueType *o) override { calls[0]++; host_op(0, i, o); }
    void DevPrecond(const ValueType *i, ValueType *o) override { calls[0]++; dev_op(0, i, o); }
    void HostPrecond_rhs(const ValueType *i, ValueType *o) override { calls[4]++; host_op(1, i, o); }
    void HostPrecond_right(const ValueType *i, ValueType *o) override { calls[2]++; host_op(1, i, o); }
    void HostPrecond_left(const ValueType *i, ValueType *o) override { calls[1]++; host_op(1, i, o); }
    void HostPrecond_starting_value(const ValueType *i, ValueType *o) override { calls[3]++; host_op(2, i, o); }
    void DevPrecond_rhs(float *i, float *o) override { calls[4]++; dev_op(1, i, o); }
    void DevPrecond_right(float *i, float *o) override { calls[2]++; dev_op(1, i, o); }
    void DevPrecond_left(float *i, float *o) override { calls[1]++; dev_op(1, i, o); }
    void DevPrecond_starting_value(float *i, float *o) override { calls[3]++; dev_op(2, i, o); }
};

template <class T>
T *to_dev(const std::vector<T> &h)
{
    void *p = nullptr;
    check(hipMalloc(&p, sizeof(T) * (h.empty() ? 1 : h.size())), "hipMalloc");
    if (!h.empty()) check(hipMemcpy(p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice), "H2D");
    return static_cast<T *>(p);
}

// the plug-in as a C-ABI operator (gg_set_precond_user): the left engine's DevPrecond
int jacobi_fn(void *ctx, int op, const float *in, float *out, int n)
{
    (void)op;
    (void)n;
    static_cast<Jacobi *>(ctx)->DevPrecond(in, out);
    return 0;
}

constexpr int kSteps = 100;

int transient(int n, int nnz, int m, int max_it, float tol, const std::vector<int> &rp, const std::vector<int> &ci,
              const std::vector<float> &val, const std::vector<float> &b, const std::vector<float> &x0, Jacobi &P,
              const char *outp)
{
    float *d_val = to_dev(val), *d_x = to_dev(x0), *d_b = to_dev(b);
    int *d_rp = to_dev(rp), *d_ci = to_dev(ci);
    SpMatrixGPU Sparse;
    std::memset(&Sparse, 0, sizeof Sparse);
    Sparse.d_val = d_val;
    Sparse.d_indices = d_ci;
    Sparse.d_rowIndices = d_rp;
    SpMatrix spm;
    std::memset(&spm, 0, sizeof spm);
    spm.numRows = spm.numCols = n;
    spm.numNZEntries = nnz;
    dim3 grid(1), block(256);
    GMRES_GPU_Data ws;
    ws.Initilize(m, n);
    std::vector<float> bt(n);
    auto rhs = [&](int t) {
        for (int i = 0; i < n; i++) bt[i] = b[i] * (1.0f + 0.01f * (float)t);
        check(hipMemcpy(d_b, bt.data(), sizeof(float) * n, hipMemcpyHostToDevice), "H2D b");
    };
    using clk = std::chrono::steady_clock;
    // step 0 sets the engine up (the caller's first call); the timed steps follow
    rhs(0);
    int ret = GMRES_GPU_tran(&Sparse, &spm, &grid, &block, d_x, d_b, n, m, max_it, tol, P, ws);
    const long long setups0 = gg_set_matrix_count();
    auto t0 = clk::now();
    for (int t = 1; t <= kSteps; t++) {
        rhs(t);
        ret = GMRES_GPU_tran(&Sparse, &spm, &grid, &block, d_x, d_b, n, m, max_it, tol, P, ws);
    }
    const double tran_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count() / kSteps;
    const int setups = (int)(gg_set_matrix_count() - setups0);
    std::vector<float> xt(n), xc(n);
    check(hipMemcpy(xt.data(), d_x, sizeof(float) * n, hipMemcpyDeviceToHost), "D2H x");
    // the C ABI alone: one solver, set up once, the same steps
    check(hipMemcpy(d_x, x0.data(), sizeof(float) * n, hipMemcpyHostToDevice), "H2D x");
    int dev = 0;
    check(hipGetDevice(&dev), "device");
    gg_solver *s = nullptr;
    std::vector<double> dv(val.begin(), val.end());
    if (gg_create(dev, &s) != GG_OK || gg_set_matrix(s, n, rp.data(), ci.data(), dv.data()) != GG_OK ||
        gg_set_precond_user(s, 0, jacobi_fn, &P) != GG_OK) {
        std::fprintf(stderr, "engine_driver: C ABI setup: %s\n", gg_last_error());
        return 3;
    }
    gg_options o{m, max_it, (double)tol, 0};
    gg_result res{};
    rhs(0);
    (void)gg_solve_device_f32(s, d_b, d_x, &o, &res);
    t0 = clk::now();
    for (int t = 1; t <= kSteps; t++) {
        rhs(t);
        if (gg_solve_device_f32(s, d_b, d_x, &o, &res) < 0) {
            std::fprintf(stderr, "engine_driver: gg_solve_device_f32: %s\n", gg_last_error());
            return 3;
        }
    }
    const double direct_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count() / kSteps;
    check(hipMemcpy(xc.data(), d_x, sizeof(float) * n, hipMemcpyDeviceToHost), "D2H x");
    gg_destroy(s);
    for (void *p : {(void *)d_val, (void *)d_x, (void *)d_b, (void *)d_rp, (void *)d_ci}) (void)hipFree(p);
    FILE *out = std::fopen(outp, "wb");
    if (!out) return 2;
    std::fwrite(&ret, sizeof ret, 1, out);
    std::fwrite(&setups, sizeof setups, 1, out);
    std::fwrite(&tran_ms, sizeof tran_ms, 1, out);
    std::fwrite(&direct_ms, sizeof direct_ms, 1, out);
    std::fwrite(xt.data(), sizeof(float), n, out);
    std::fwrite(xc.data(), sizeof(float), n, out);
    std::fclose(out);
    return 0;
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: engine_driver IN OUT\n");
        return 2;
    }
    g_in = std::fopen(argv[1], "rb");
    if (!g_in) return 2;
    const int mode = rd<int>(1)[0], n = rd<int>(1)[0], nnz = rd<int>(1)[0], m = rd<int>(1)[0];
    int max_it = rd<int>(1)[0];
    float tol = rd<float>(1)[0];
    std::vector<int> rp = rd<int>(n + 1), ci = rd<int>(nnz);
    std::vector<float> val = rd<float>(nnz), b = rd<float>(n), x = rd<float>(n);
    std::fclose(g_in);

    MySpMatrix A;                                   // the caller's host CSR (mySpMatrix)
    std::memset(&A, 0, sizeof A);
    A.isCSR = 1;
    A.numRows = A.numCols = n;
    A.numNZEntries = nnz;
    A.val = val.data();
    A.indices = ci.data();
    A.rowIndices = rp.data();
    Jacobi P;
    P.Initilize(A);

    if (mode == 4) return transient(n, nnz, m, max_it, tol, rp, ci, val, b, x, P, argv[2]);
    int ret = 1;
    if (mode == 3) {                                // host engine, host arrays
        ret = GMRESilu(val.data(), rp.data(), ci.data(), x.data(), b.data(), n, m, &max_it, &tol, P);
    } else {
        float *d_val = to_dev(val), *d_x = to_dev(x), *d_b = to_dev(b);
        int *d_rp = to_dev(rp), *d_ci = to_dev(ci);
        SpMatrixGPU Sparse;
        std::memset(&Sparse, 0, sizeof Sparse);
        Sparse.d_val = d_val;
        Sparse.d_indices = d_ci;
        Sparse.d_rowIndices = d_rp;
        SpMatrix spm;
        std::memset(&spm, 0, sizeof spm);
        spm.numRows = spm.numCols = n;
        spm.numNZEntries = nnz;
        dim3 grid(1), block(256);
        if (mode == 0) {
            ret = GMRES_GPU(&Sparse, &spm, &grid, &block, d_x, d_b, n, m, &max_it, &tol, P);
        } else if (mode == 1) {
            GMRES_GPU_Data ws;
            ws.Initilize(m, n);
            ret = GMRES_GPU_tran(&Sparse, &spm, &grid, &block, d_x, d_b, n, m, max_it, tol, P, ws);
        } else {
            ret = GMRESilu_GPU(d_val, d_rp, d_ci, nnz, d_x, d_b, n, m, &max_it, &tol, P);
        }
        check(hipMemcpy(x.data(), d_x, sizeof(float) * n, hipMemcpyDeviceToHost), "D2H x");
        for (void *p : {(void *)d_val, (void *)d_x, (void *)d_b, (void *)d_rp, (void *)d_ci}) (void)hipFree(p);
    }
    FILE *out = std::fopen(argv[2], "wb");
    if (!out) return 2;
    std::fwrite(&ret, sizeof ret, 1, out);
    std::fwrite(&max_it, sizeof max_it, 1, out);
    std::fwrite(&tol, sizeof tol, 1, out);
    std::fwrite(P.calls, sizeof(int), 5, out);
    std::fwrite(x.data(), sizeof(float), n, out);
    std::fclose(out);
    return 0;
}
