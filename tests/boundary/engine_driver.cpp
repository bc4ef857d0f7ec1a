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
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>

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
