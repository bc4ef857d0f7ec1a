// interface_pg.cpp -- libggmres.so implementation of the reference's PG solver
// boundary classes (include/gmres_interface_pg.h), forwarding to the C ABI.
//
// Reference: src/gmres_interface_pg.cu:9-163.  Ownership as in the reference:
// A's host arrays and the factor arrays are borrowed (copied to HBM here, the
// caller frees them, src/mna_solve_gpu_gmres.cpp:852-870); xgmres_h / rhs_h
// are malloc'd here and freed by the destructor.  The fp32 device mirrors
// d_val / d_rowPtr / d_colIdx / xgmres_d / rhs_d of the reference are not
// needed by the fp64 engine and are left null (no caller reads them).
// Errors: the reference exits or asserts; here an error is printed, Precond
// stays null and the solve methods return 1 ("Failed to converge.").
// Engines as in the reference: GMRES_dev_PG runs the device engine (gg_solve,
// the split preconditioner on the GPU); GMRES_host_PG runs the HOST engine
// (csrc/host/gmres_host.cpp: GMRESilu with HostPrecond_*, fp64 on the CPU) --
// Precond holds both (PGEngines).
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <hip/hip_runtime.h>

#include "gmres_interface_pg.h"
#include "ggmres.h"
#include "host/gmres_host.h"

// ---- the layout is the ABI (x86-64, LP64) --------------------------------------
static_assert(sizeof(MySpMatrix) == 64 && offsetof(MySpMatrix, val) == 40 &&
                  offsetof(MySpMatrix, rowIndices) == 56,
              "MySpMatrix layout differs from src/SpMV.h:57-84");
static_assert(sizeof(MySpMatrixDouble) == 64 && offsetof(MySpMatrixDouble, val) == 40,
              "MySpMatrixDouble layout differs from src/SpMV.h:88-102");
static_assert(offsetof(gmresInterfacePGfloat, nnz) == 4 &&
                  offsetof(gmresInterfacePGfloat, h_val) == 8 &&
                  offsetof(gmresInterfacePGfloat, d_val) == 32 &&
                  offsetof(gmresInterfacePGfloat, xgmres_h) == 72 &&
                  offsetof(gmresInterfacePGfloat, rhs_h) == 80 &&
                  offsetof(gmresInterfacePGfloat, Precond) == 104 &&
                  offsetof(gmresInterfacePGfloat, max_it) == 112 &&
                  offsetof(gmresInterfacePGfloat, tol) == 116 &&
                  sizeof(gmresInterfacePGfloat) == 120,
              "gmresInterfacePGfloat layout differs from src/gmres_interface_pg.h:38-73");
static_assert(offsetof(gmresInterfacePG, h_val) == 8 && offsetof(gmresInterfacePG, xgmres_h) == 48 &&
                  offsetof(gmresInterfacePG, rhs_h) == 56 && offsetof(gmresInterfacePG, Precond) == 64 &&
                  offsetof(gmresInterfacePG, max_it) == 72 && offsetof(gmresInterfacePG, tol) == 76 &&
                  sizeof(gmresInterfacePG) == 80,
              "gmresInterfacePG layout differs from src/gmres_interface_pg.h:5-36");

namespace {

constexpr int kRestart = 32;          // const int restart (src/defs.h:11)
constexpr int kMaxIterPG = 10000;     // src/gmres_interface_pg.cu:66,114
constexpr int kMaxIterDefs = 60000;   // const int max_iter (src/defs.h:11)
constexpr double kTolPG = 1e-7;       // gmres_tol_global (src/gmres_interface_pg.cu:7)

template <class T>
std::vector<double> promote(const T *p, int n)
{
    std::vector<double> d(n);
    for (int i = 0; i < n; i++) d[i] = (double)p[i];
    return d;
}

// what Precond points at: the device solver and the host engine's operands
struct PGEngines {
    gg_solver *dev = nullptr;
    gg::HostSplitEngine host;
    ~PGEngines() { gg_destroy(dev); }
};

template <class ScaleT>
gg_solver *build_solver(MySpMatrix *A, MySpMatrixDouble *L, MySpMatrixDouble *U, MySpMatrix *middle,
                        MySpMatrix *prow, MySpMatrix *pcol, const ScaleT *lscale, const ScaleT *rscale)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    gg_solver *s = nullptr;
    int rc = gg_create(dev, &s);
    const int n = A->numRows;
    if (rc == GG_OK) {
        std::vector<double> av = promote(A->val, A->rowIndices[n]);
        rc = gg_set_matrix(s, n, A->rowIndices, A->indices, av.data());
    }
    if (rc == GG_OK) {
        std::vector<double> mid = promote(middle->val, n);
        std::vector<double> ls = promote(lscale, n), rs = promote(rscale, n);
        rc = gg_set_precond_split(s, L->rowIndices, L->indices, L->val, U->rowIndices, U->indices,
                                  U->val, mid.data(), prow->indices, pcol->indices, ls.data(),
                                  rs.data());
    }
    if (rc != GG_OK) {
        std::fprintf(stderr, "gmresInterfacePG::setPrecondPG: %s (%s)\n", gg_strerror(rc),
                     gg_last_error());
        gg_destroy(s);
        return nullptr;
    }
    return s;
}

// both engines for one interface object
template <class ScaleT>
void *build_engines(MySpMatrix *A, MySpMatrixDouble *L, MySpMatrixDouble *U, MySpMatrix *middle,
                    MySpMatrix *prow, MySpMatrix *pcol, const ScaleT *lscale, const ScaleT *rscale)
{
    // (the host engine needs no device: a CPU-only caller of GMRES_host_PG keeps
    // working when the device set-up failed -- only GMRES_dev_PG then fails)
    PGEngines *e = new PGEngines;
    e->dev = build_solver(A, L, U, middle, prow, pcol, lscale, rscale);
    gg::HostSplitEngine &h = e->host;
    const int n = A->numRows;
    h.n = n;
    h.arp.assign(A->rowIndices, A->rowIndices + n + 1);
    h.aci.assign(A->indices, A->indices + h.arp[n]);
    h.av = promote(A->val, h.arp[n]);
    h.lrp.assign(L->rowIndices, L->rowIndices + n + 1);
    h.lci.assign(L->indices, L->indices + h.lrp[n]);
    h.lv.assign(L->val, L->val + h.lrp[n]);
    h.urp.assign(U->rowIndices, U->rowIndices + n + 1);
    h.uci.assign(U->indices, U->indices + h.urp[n]);
    h.uv.assign(U->val, U->val + h.urp[n]);
    h.mid = promote(middle->val, n);
    h.prow.assign(prow->indices, prow->indices + n);
    h.pcol.assign(pcol->indices, pcol->indices + n);
    h.ls = promote(lscale, n);
    h.rs = promote(rscale, n);
    return e;
}

// the host engine with fp32 I/O at the boundary; returns the reference's 0/1
int solve_host_f32(void *handle, int n, const float *rhs, float *x, int max_iter, double tol, int *it_out,
                   float *tol_out)
{
    PGEngines *e = (PGEngines *)handle;
    if (!e) {
        std::printf("Failed to converge.\n");
        return 1;
    }
    std::vector<double> b = promote(rhs, n), xd = promote(x, n);
    int it = max_iter;
    double t = tol;
    const int rc = gg::gmres_split_host(e->host, b.data(), xd.data(), kRestart, &it, &t, nullptr);
    for (int i = 0; i < n; i++) x[i] = (float)xd[i];
    if (it_out) *it_out = it;
    if (tol_out) *tol_out = (float)t;
    if (rc != 0) std::printf("Failed to converge.\n");
    return rc;
}

// solve with fp32 I/O at the boundary; returns the reference's 0/1
int solve_f32(void *handle, int n, const float *rhs, float *x, int max_iter, double tol,
              int *it_out, float *tol_out)
{
    gg_solver *s = handle ? ((PGEngines *)handle)->dev : nullptr;
    if (!s) {
        std::printf("Failed to converge.\n");
        return 1;
    }
    std::vector<double> b = promote(rhs, n), xd = promote(x, n);
    gg_options o{kRestart, max_iter, tol, 0};
    gg_result r{};
    int rc = gg_solve(s, b.data(), xd.data(), &o, &r);
    if (rc < 0) {
        std::fprintf(stderr, "GMRES: %s (%s)\n", gg_strerror(rc), gg_last_error());
        std::printf("Failed to converge.\n");
        return 1;
    }
    for (int i = 0; i < n; i++) x[i] = (float)xd[i];
    if (it_out) *it_out = r.iters;
    if (tol_out) *tol_out = (float)r.relres;
    if (rc != 0) std::printf("Failed to converge.\n");
    return rc;
}

}  // namespace

// ----------------------------------------------------------- gmresInterfacePG
void gmresInterfacePG::setPrecondPG(MySpMatrix *A, MySpMatrixDouble *PrLeft, MySpMatrixDouble *PrRight,
                                    MySpMatrix *PrMiddle, MySpMatrix *PrPermRow, MySpMatrix *PrPermCol,
                                    MySpMatrixDouble *PrLscale, MySpMatrixDouble *PrRscale)
{
    matrixSize = A->numRows;
    h_val = A->val;
    h_rowPtr = A->rowIndices;
    h_colIdx = A->indices;
    x_h = x_d = nullptr;
    xgmres_h = (float *)std::malloc(matrixSize * sizeof(float));
    rhs_h = (float *)std::malloc(matrixSize * sizeof(float));
    max_it = kMaxIterPG;
    tol = (float)kTolPG;
    Precond = build_engines(A, PrLeft, PrRight, PrMiddle, PrPermRow, PrPermCol, PrLscale->val,
                            PrRscale->val);
}

int gmresInterfacePG::GMRES_host_PG()
{
    max_it = kMaxIterPG;
    tol = (float)kTolPG;
    return solve_host_f32(Precond, matrixSize, rhs_h, xgmres_h, max_it, kTolPG, &max_it, &tol);
}

gmresInterfacePG::~gmresInterfacePG()
{
    std::free(xgmres_h);
    std::free(rhs_h);
    delete (PGEngines *)Precond;
}

// ------------------------------------------------------ gmresInterfacePGfloat
void gmresInterfacePGfloat::setPrecondPG(MySpMatrix *A, MySpMatrixDouble *PrLeft,
                                         MySpMatrixDouble *PrRight, MySpMatrix *PrMiddle,
                                         MySpMatrix *PrPermRow, MySpMatrix *PrPermCol,
                                         MySpMatrix *PrLscale, MySpMatrix *PrRscale)
{
    matrixSize = A->numRows;
    h_val = A->val;
    h_rowPtr = A->rowIndices;
    h_colIdx = A->indices;
    nnz = h_rowPtr[matrixSize];
    d_val = nullptr;
    d_rowPtr = d_colIdx = nullptr;
    x_h = x_d = nullptr;
    xgmres_d = rhs_d = nullptr;
    xgmres_h = (float *)std::malloc(matrixSize * sizeof(float));
    rhs_h = (float *)std::malloc(matrixSize * sizeof(float));
    max_it = kMaxIterPG;
    tol = (float)kTolPG;
    Precond = build_engines(A, PrLeft, PrRight, PrMiddle, PrPermRow, PrPermCol, PrLscale->val,
                            PrRscale->val);
}

int gmresInterfacePGfloat::GMRES_host_PG()
{
    // the reference solves with LOCAL max_it / tol copies (src/gmres_interface_pg.cu:88-90):
    // the members are not updated
    int it = 0;
    float t = 0.f;
    return solve_host_f32(Precond, matrixSize, rhs_h, xgmres_h, kMaxIterDefs, kTolPG, &it, &t);
}

int gmresInterfacePGfloat::GMRES_dev_PG()
{
    max_it = kMaxIterPG;
    tol = (float)kTolPG;
    return solve_f32(Precond, matrixSize, rhs_h, xgmres_h, max_it, kTolPG, &max_it, &tol);
}

gmresInterfacePGfloat::~gmresInterfacePGfloat()
{
    std::free(xgmres_h);
    std::free(rhs_h);
    delete (PGEngines *)Precond;
}
