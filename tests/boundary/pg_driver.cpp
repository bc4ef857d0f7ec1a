// pg_driver.cpp -- a stand-in for the reference's caller of the PG solver
// classes (src/mna_solve_gpu_gmres.cpp:507-545, 608-621), compiled with g++ and
// linked against libggmres.so exactly as mna_solve_gpu_gmres.o would be: it
// includes only gmres_interface_pg.h, fills MySpMatrix / MySpMatrixDouble the
// way the reference's feeders do (index_list2csrMySpMatrix, ILUPPvec2csrMySpMatrix,
// ILUPPmat2csrMySpMatrixDouble in ROW orientation: src/mna_solve_gpu_gmres.cpp:26-188),
// calls setPrecondPG, writes rhs_h / xgmres_h directly, and solves a sequence
// of right-hand sides with the previous solution as the warm start (the
// transient loop's use of one interface object).
//
//   pg_driver IN OUT
// IN  (little-endian): int32 mode (0: gmresInterfacePGfloat::GMRES_dev_PG,
//     1: gmresInterfacePGfloat::GMRES_host_PG, 2: gmresInterfacePG::GMRES_host_PG),
//     n, nnzA, nnzL, nnzU, nsteps; A rp[n+1] ci[nnzA] float val[nnzA];
//     L rp ci double val; U rp ci double val; float middle[n]; int32 perm_row[n],
//     perm_col[n]; lscale[n], rscale[n] (float for modes 0-1, double for 2);
//     float x0[n]; float rhs[nsteps][n]
// OUT per step: int32 return code, int32 max_it, float tol, float x[n]
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "gmres_interface_pg.h"

namespace {

FILE *g_in;

template <class T>
std::vector<T> rd(size_t count)
{
    std::vector<T> v(count);
    if (count && std::fread(v.data(), sizeof(T), count, g_in) != count) {
        std::fprintf(stderr, "pg_driver: short input\n");
        std::exit(2);
    }
    return v;
}

template <class T>
T *heap(const std::vector<T> &v)            // the feeders malloc their arrays
{
    T *p = (T *)std::malloc(sizeof(T) * (v.empty() ? 1 : v.size()));
    for (size_t k = 0; k < v.size(); k++) p[k] = v[k];
    return p;
}

// index_list2csrMySpMatrix (src/mna_solve_gpu_gmres.cpp:26-47)
void index_list(MySpMatrix *M, const std::vector<int> &perm, int n)
{
    M->isCSR = 1;
    M->numRows = M->numCols = M->numNZEntries = n;
    M->rowIndices = (int *)std::malloc((n + 1) * sizeof(int));
    M->indices = (int *)std::malloc(n * sizeof(int));
    M->val = (float *)std::malloc(n * sizeof(float));
    for (int i = 0; i < n; i++) {
        M->val[i] = 1.0f;
        M->indices[i] = perm[i];
    }
    for (int i = 0; i <= n; i++) M->rowIndices[i] = i;
}

// ILUPPvec2csrMySpMatrix(Double) (:132-188)
template <class S, class T>
void vec(S *M, const std::vector<T> &v, int n)
{
    M->isCSR = 1;
    M->numRows = M->numCols = M->numNZEntries = n;
    M->rowIndices = (int *)std::malloc((n + 1) * sizeof(int));
    M->indices = (int *)std::malloc(n * sizeof(int));
    M->val = heap(v);
    for (int j = 0; j <= n; j++) M->rowIndices[j] = j;
    for (int i = 0; i < n; i++) M->indices[i] = i;
}

// a CSR matrix as ILUPPmat2csrMySpMatrix(Double) leaves a ROW-oriented one
template <class S, class T>
void mat(S *M, int n, int nnz, const std::vector<int> &rp, const std::vector<int> &ci, const std::vector<T> &v)
{
    M->isCSR = 1;
    M->numRows = M->numCols = n;
    M->numNZEntries = nnz;
    M->rowIndices = heap(rp);
    M->indices = heap(ci);
    M->val = heap(v);
}

template <class S>
void release(S *M)                           // mySpMatrixFree: the caller frees
{
    std::free(M->rowIndices);
    std::free(M->indices);
    std::free(M->val);
}

template <class I, class ScaleT>
int run(FILE *out, int mode, int n, int nsteps, MySpMatrix &A, MySpMatrixDouble &L, MySpMatrixDouble &U,
        MySpMatrix &mid, MySpMatrix &prow, MySpMatrix &pcol, ScaleT &ls, ScaleT &rs,
        const std::vector<float> &x0, const std::vector<float> &rhs)
{
    I itf;
    itf.setPrecondPG(&A, &L, &U, &mid, &prow, &pcol, &ls, &rs);
    if (!itf.Precond) return 3;
    for (int i = 0; i < n; i++) itf.xgmres_h[i] = x0[i];
    for (int k = 0; k < nsteps; k++) {
        for (int i = 0; i < n; i++) itf.rhs_h[i] = rhs[(size_t)k * n + i];
        int rc;
        if constexpr (std::is_same<I, gmresInterfacePGfloat>::value) {
            rc = mode == 0 ? itf.GMRES_dev_PG() : itf.GMRES_host_PG();
        } else {
            rc = itf.GMRES_host_PG();
        }
        std::fwrite(&rc, sizeof(int), 1, out);
        std::fwrite(&itf.max_it, sizeof(int), 1, out);
        std::fwrite(&itf.tol, sizeof(float), 1, out);
        std::fwrite(itf.xgmres_h, sizeof(float), n, out);
    }
    return 0;
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: pg_driver IN OUT\n");
        return 2;
    }
    g_in = std::fopen(argv[1], "rb");
    FILE *out = std::fopen(argv[2], "wb");
    if (!g_in || !out) return 2;
    const std::vector<int> hdr = rd<int>(6);
    const int mode = hdr[0], n = hdr[1], nnzA = hdr[2], nnzL = hdr[3], nnzU = hdr[4], nsteps = hdr[5];
    MySpMatrix A{}, mid{}, prow{}, pcol{};
    MySpMatrixDouble L{}, U{};
    {
        auto rp = rd<int>(n + 1), ci = rd<int>(nnzA);
        auto v = rd<float>(nnzA);
        mat(&A, n, nnzA, rp, ci, v);
    }
    {
        auto rp = rd<int>(n + 1), ci = rd<int>(nnzL);
        auto v = rd<double>(nnzL);
        mat(&L, n, nnzL, rp, ci, v);
    }
    {
        auto rp = rd<int>(n + 1), ci = rd<int>(nnzU);
        auto v = rd<double>(nnzU);
        mat(&U, n, nnzU, rp, ci, v);
    }
    vec(&mid, rd<float>(n), n);
    index_list(&prow, rd<int>(n), n);
    index_list(&pcol, rd<int>(n), n);
    int rc;
    if (mode == 2) {
        MySpMatrixDouble ls{}, rs{};
        vec(&ls, rd<double>(n), n);
        vec(&rs, rd<double>(n), n);
        auto x0 = rd<float>(n);
        auto rhs = rd<float>((size_t)nsteps * n);
        rc = run<gmresInterfacePG>(out, mode, n, nsteps, A, L, U, mid, prow, pcol, ls, rs, x0, rhs);
        release(&ls);
        release(&rs);
    } else {
        MySpMatrix ls{}, rs{};
        vec(&ls, rd<float>(n), n);
        vec(&rs, rd<float>(n), n);
        auto x0 = rd<float>(n);
        auto rhs = rd<float>((size_t)nsteps * n);
        rc = run<gmresInterfacePGfloat>(out, mode, n, nsteps, A, L, U, mid, prow, pcol, ls, rs, x0, rhs);
        release(&ls);
        release(&rs);
    }
    for (MySpMatrix *M : {&A, &mid, &prow, &pcol}) release(M);
    for (MySpMatrixDouble *M : {&L, &U}) release(M);
    std::fclose(out);
    std::fclose(g_in);
    return rc;
}
