/*
 * oracle.h -- fp64 CPU restatement of the reference GPU-GMRES hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gpu-gmres_amd/, include/)
 * links, loads or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, as the checker / CPU baseline.
 *
 * Every routine restates one reference routine operation-for-operation in
 * double precision (the reference computes in float).
 * Reference paths are relative to the upstream tree (sheldonucr/GPU-GMRES).
 *
 * Parity status: the reference's own tests pin no GMRES residual history
 * (SURVEY.md Sec. 4, 8(c)); building/running the reference was refused in
 * this environment.  The restatement is therefore
 * checked against the reference's data fixtures (cusp laplacian/random
 * matrices, sherman1) through independent numpy/scipy computations
 * (tests/golden/make_golden.py) -- see DESIGN.md "Oracle".
 */
#ifndef GG_ORACLE_H_
#define GG_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* y = A x   (computeSpMV, src/SpMV_compute.cpp:19-36) */
void orc_spmv(int n, const int *rp, const int *ci, const double *v,
              const double *x, double *y);

/* r = -1*A*x + 1*b   (sgemv, src/gmres.cu:77-88) */
void orc_residual(int n, const int *rp, const int *ci, const double *v,
                  const double *x, const double *b, double *r);

/* Left-looking ILU(0) (leftILU, src/leftILU.cu:27-336, CPU column kernel
 * cpuSequentialTriSolve :769-825, level order generateLevel :339-368,
 * final split splitLU_csr :481-541).  L: strictly-lower entries + unit diag
 * stored LAST per row; U: entries col>=row (diag first for sorted input).
 * Outputs are malloc'd; release with orc_free.  Returns 0. */
/* the factored matrix of orc_ilu0 before its split (A's sorted CSR order) */
int orc_ilu0_values(int n, const int *rp, const int *ci, const double *v, double *out);
int orc_ilu0(int n, const int *rp, const int *ci, const double *v,
             int *l_rp, int **l_ci, double **l_v,
             int *u_rp, int **u_ci, double **u_v);

/* ILU(k) -- ITSOL lofC + ilukC (src/iluk.cpp:56-334) restated in double.
 * Output layout matches orc_ilu0 (L unit diag last, U diag first + strict
 * upper sorted ascending).  Returns 0, or -2 on a zero pivot (iluk.cpp:175). */
int orc_iluk(int lofM, int n, const int *rp, const int *ci, const double *v,
             int *l_rp, int **l_ci, double **l_v,
             int *u_rp, int **u_ci, double **u_v);

void orc_free(void *p);
/* threads the OpenMP build (liboracle_mt.so) runs its loops on; 1 for the checker */
int orc_threads(void);

/* x = (LU)^-1 y  (LUSolve_ignoreZero, src/SpMV_compute.cpp:92-136) */
void orc_set_div_mode(int mul_l, int mul_u);
void orc_set_fma_tail(int tail);
void orc_set_orth(int cgs2);
void orc_lusolve(int n, const int *l_rp, const int *l_ci, const double *l_v,
                 const int *u_rp, const int *u_ci, const double *u_v,
                 const double *y, double *x);

/* Split (ILU++/PG) preconditioner maps, MyILUPP::HostPrecond_*
 * (src/preconditioner.cu:1074-1137).  L: non-unit, diag last; U: diag first. */
typedef struct {
    int n;
    const int *l_rp, *l_ci; const double *l_v;
    const int *u_rp, *u_ci; const double *u_v;
    const double *middle, *lscale, *rscale;
    const int *perm_row, *perm_col;
} orc_split_t;
void orc_split_left(const orc_split_t *p, const double *in, double *out);
void orc_split_right(const orc_split_t *p, const double *in, double *out);
void orc_split_start(const orc_split_t *p, const double *in, double *out);

/* Dot-product summation order used by the GMRES restatements: blocked = 0
 * is the reference CPU engine's serial loop (default); blocked = 1 restates
 * the device kernels' reduction tree over a laid-out vector (see oracle.c). */
void orc_set_dot_order(int blocked, long long ppad, int G, const long long *lay2nat);
void orc_set_dot_order_shards(int nseg, const long long *seglen, int G, const long long *lay2nat);

/* Givens (src/gmres.cu:192-216) */
void orc_apply_rot(double *dx, double *dy, double cs, double sn);
void orc_gen_rot(double dx, double dy, double *cs, double *sn);

/* GMRES_leftILU0 (src/gmres.cu:566-717).  x: in x0 / out solution.
 * *max_iter in/out (reference semantics), *tol in/out.
 * hist receives [beta0/normb, per-iteration |s[i+1]|/normb ...,
 * beta/normb at each restart ...]; *hist_len its length (capped at hist_cap).
 * *inner_iters: number of Arnoldi iterations actually performed.
 * Returns 0 converged, 1 not converged. */
int orc_gmres_left(int n, const int *rp, const int *ci, const double *v,
                   const int *l_rp, const int *l_ci, const double *l_v,
                   const int *u_rp, const int *u_ci, const double *u_v,
                   const double *b, double *x, int m, int *max_iter, double *tol,
                   double *hist, int hist_cap, int *hist_len, int *inner_iters);

/* GMRESilu (src/gmres.cu:2069-2252) with the split preconditioner above. */
int orc_gmres_split(int n, const int *rp, const int *ci, const double *v,
                    const orc_split_t *p,
                    const double *b, double *x, int m, int *max_iter, double *tol,
                    double *hist, int hist_cap, int *hist_len, int *inner_iters);

/* Transient step (src/mna_solve_gpu_gmres.cpp:564-647).  PULSE value of a
 * source at time index it (gen_PULSEut_kernel, src/kernels.cu:223-245);
 * q = {vlo, vhi, td, tr, tf, tw, tp}. */
double orc_pulse(const double *q, int it, double h);
double orc_pwl(const double *tv, int np, int it, double h);
/* w = B u + (C/h) x formed as the driver does: w = 0; w += B u (cs_dl_gaxpy,
 * B incidence: source k adds +1 * u[k] at row src_node[k], k ascending);
 * xnr = 0; xnr += diag(cdiag) x; w += xnr. */
void orc_gaxpy_csc(int ncol, const long *p, const long *i, const double *ax, const double *x, double *y);
void orc_transient_rhs(int n, int nsrc, const int *src_node, const double *u,
                       const double *cdiag, const double *x, double *w);

/* sharded solve pieces (oracle/dd.py) */
void orc_canon_trsv(int n, int lower, const int *rp, const int *ci, const double *v,
                    const double *d, const double *b, double *x);
void orc_sub_seq(int n, const int *rp, const int *ci, const double *v, const double *x,
                 const double *in, double *out);

#ifdef __cplusplus
}
#endif
#endif
