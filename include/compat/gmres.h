/*
 * compat/gmres.h -- the reference's GMRES engine entry points that take the
 * Preconditioner plug-in (src/gmres.h:82-112, 356-398; include guard included),
 * exported by libggmres.so with the reference's C++ signatures (Itanium
 * mangling, g++ / hipcc alike):
 *
 *   GMRES_GPU(SpMatrixGPU*, SpMatrix*, dim3*, dim3*, float *d_x, const float *d_b,
 *             n, m, int *max_iter, float *tol, Preconditioner&)   src/gmres.cu:2567-2732
 *   GMRES_GPU_tran(..., max_iter, tol, Preconditioner&, GMRES_GPU_Data&)
 *                                                                src/gmres.cu:2736-2827
 *   GMRESilu_GPU(float *val, int *rowIndices, int *indices, int nnz, float *x,
 *                float *b, n, m, int *max_iter, float *tol, Preconditioner&)
 *                                                                src/gmres.cu:2254-2446
 *   GMRESilu(host arrays ..., Preconditioner&)                   src/gmres.cu:2069-2252
 *
 * Semantics as the reference: left-preconditioned GMRES(m) calling
 * preconditioner.DevPrecond (GMRES_GPU, _tran), the split engine calling
 * DevPrecond_rhs / _left / _right / _starting_value (GMRESilu_GPU; GMRESilu
 * calls the Host* methods with host arrays); CSR and vectors in fp32 device
 * memory (host memory for GMRESilu); return 0 converged / 1 not; on return
 * *max_iter = iterations used, *tol = relative residual achieved.  The solve
 * itself runs the library's fp64 engine (ggmres.h, gg_set_precond_user): the
 * fp32 inputs are promoted, every preconditioner call sees fp32 arrays, x is
 * rounded to fp32 at the end.  grid / block (the reference's SpMV launch shape)
 * are accepted and ignored.  Errors: a message on stderr and return 1.
 */
#ifndef _GMRES_H_
#define _GMRES_H_

#include <hip/hip_runtime_api.h>   /* dim3 */

#include "SpMV.h"
#include "preconditioner.h"

/* src/gmres.h:82-112: the workspace GMRES_GPU_tran borrows (kept here for the
 * layout; libggmres's engine keeps its own) */
class GMRES_GPU_Data {
public:
    int numRows;
    float *s, *cs, *sn, *H;
    float *d_r, *d_rr, *d_bb, *d_temp;
    float *d_v, *d_w, *d_ww;

    void Initilize(const int m, const int n)
    {
        numRows = n;
        s = new float[m + 1];
        cs = new float[m + 1];
        sn = new float[m + 1];
        H = new float[(size_t)m * (m + 1)];
        d_r = d_rr = d_bb = d_temp = d_v = d_w = d_ww = nullptr;
    }
    ~GMRES_GPU_Data()
    {
        delete[] s;
        delete[] cs;
        delete[] sn;
        delete[] H;
    }
};

int GMRES_GPU(SpMatrixGPU *Sparse, SpMatrix *spm, dim3 *grid, dim3 *block,
              float *d_x, const float *d_b, const int n,
              const int m, int *max_iter, float *tol,
              Preconditioner &preconditioner);

int GMRES_GPU_tran(SpMatrixGPU *Sparse, SpMatrix *spm, dim3 *grid, dim3 *block,
                   float *d_x, const float *d_b, const int n,
                   const int m, const int max_iter,
                   const float tol,
                   Preconditioner &preconditioner,
                   GMRES_GPU_Data &gmres_gpu_data);

int GMRESilu(const float *val, const int *rowIndices, const int *indices,
             float *x, const float *b, const int n,
             const int m, int *max_iter, float *tol,
             Preconditioner &preconditioner);

int GMRESilu_GPU(float *val, int *rowIndices, int *indices, int nnz,
                 float *x, float *b, const int n,
                 const int m, int *max_iter, float *tol,
                 Preconditioner &preconditioner);

#endif /* _GMRES_H_ */
