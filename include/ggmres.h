/*
 * ggmres.h -- C ABI of the MI355X-native preconditioned GMRES solver.
 *
 * This is the drop-in boundary for the reference's hot path.
 * Every entry point below replaces one reference interface; the citation is
 * the reference file:line it stands in for (sheldonucr/GPU-GMRES):
 *
 *   gg_set_matrix          MySpMatrix / gpuMallocCpyCSRmySpM  src/SpMV.h:57-84, src/SpMV_alloc.cu:121-165
 *   gg_set_precond_ilu0    MyILU0::Initilize / leftILU        src/preconditioner.h:119-144, src/leftILU.cu:27-336
 *   gg_set_precond_ilu0_device, gg_ilu0_device_values
 *                          leftILU's device path (sparseTriSolve_V2 per level)
 *                                                               src/leftILU.cu:188-262, 650-702
 *   gg_set_precond_iluk    MyILUK::Initilize (ilukC, lofC)     src/preconditioner.cu:1659-1753, src/iluk.cpp:56-334
 *   gg_set_precond_iluk_device, gg_iluk_device_factors
 *                          the same with ilukC's numeric phase on the device  src/iluk.cpp:108-188
 *   gg_set_precond_lu      GMRES_GPU_leftILU0 L/U arguments     src/gmres.h:206-213 (src/gmres.cu:1438-1444)
 *   gg_set_precond_split   MyILUPPfloat::Initilize              src/preconditioner.cu:1205-1334
 *                          gmresInterfacePGfloat::setPrecondPG  src/gmres_interface_pg.cu:30-60
 *   gg_solve / gg_solve_device
 *                          GMRES_GPU_leftILU0 (left engine)     src/gmres.cu:1438-1696
 *                          GMRESilu_GPU (split engine)          src/gmres.cu:2254-2446
 *                          gmresInterfacePGfloat::GMRES_dev_PG  src/gmres_interface_pg.cu:110-139
 *   (no CPU twin is shipped: the reference's CPU engines GMRES_leftILU0 /
 *    GMRESilu are restated only in oracle/, which is test code)
 *   gg_spmv                cusparseScsrmv / SpMV kernel          src/gmres.cu:2351-2353, src/SpMV_kernel.cu:166-251
 *   gg_precond_apply       Preconditioner::DevPrecond_{left,right,rhs,starting_value}
 *                                                               src/preconditioner.cu:1419-1657, src/gmres.cu:1398-1428
 *
 * Conventions: CSR, 0-based int32 indices, fp64 values.  Host arrays passed
 * to gg_set_* are copied (the solver never keeps a host pointer).  Vectors
 * passed to gg_solve are host arrays in the caller's (natural) row order;
 * gg_solve_device takes device (HBM) pointers in natural order.
 *
 * Return codes: GG_OK (0) converged / success, GG_NOT_CONVERGED (1) -- the
 * reference's 0/1 convention (src/gmres.h:14-16) -- and negative errors.
 * Thread safety: one solver per host thread; solvers are independent.
 */
#ifndef GGMRES_H_
#define GGMRES_H_

#ifdef __cplusplus
extern "C" {
#endif

#define GG_ABI_VERSION 1

enum gg_status {
    GG_OK = 0,
    GG_NOT_CONVERGED = 1,
    GG_EINVAL = -1,        /* bad argument / shape                         */
    GG_EHIP = -2,          /* HIP runtime error                            */
    GG_EZEROPIVOT = -3,    /* ILU(k) zero pivot (src/iluk.cpp:175-185)     */
    GG_ENOMEM = -4,        /* device allocation failed                     */
    GG_ESTATE = -5,        /* call order (e.g. solve before set_matrix)    */
    GG_ETIMEOUT = -6,      /* a device-side wait exceeded its spin bound   */
    GG_ECOMM = -7          /* RCCL / multi-GPU error                       */
};

enum gg_precond_kind {
    GG_PRECOND_NONE = 0,
    GG_PRECOND_ILU0 = 1,   /* left, factored from A                        */
    GG_PRECOND_ILUK = 2,   /* left, factored from A                        */
    GG_PRECOND_LU = 3,     /* left, caller-supplied L,U                    */
    GG_PRECOND_SPLIT = 4,  /* ILU++/PG split: Ml = L^-1 P_r D_l^-1, Mr = D_r^-1 P_c U^-1 M */
    GG_PRECOND_USER = 5,   /* caller-supplied left operator (gg_set_precond_user)          */
    GG_PRECOND_USER_SPLIT = 6  /* caller-supplied split operators (gg_set_precond_user)     */
};

/* which operator gg_precond_apply applies */
enum gg_precond_op {
    GG_APPLY_MINV = 0,     /* left engines: (LU)^-1           (LUSolve_gpu)                    */
    GG_APPLY_LEFT = 1,     /* split: Ml   (DevPrecond_left / _rhs)                             */
    GG_APPLY_RIGHT = 2,    /* split: Mr   (DevPrecond_right)                                   */
    GG_APPLY_START = 3,    /* split: Mr^-1 (DevPrecond_starting_value)                         */
    GG_APPLY_RHS = 4       /* split: the right-hand side's Ml (DevPrecond_rhs; = LEFT for the
                              built-in split, the user's own method for GG_PRECOND_USER_SPLIT) */
};

typedef struct gg_solver gg_solver;

typedef struct gg_options {
    int restart;       /* m  (reference default 32, src/defs.h:11)                 */
    int max_iter;      /* reference semantics: in = limit                          */
    double tol;        /* relative residual target on ||M r|| / ||M b||            */
    int flags;         /* GG_SOLVE_* bits, else 0                                 */
} gg_options;

/* gg_options.flags: other solvers run on this device at the same time (one
 * solver object, stream and host thread per system, e.g. the many-RHS
 * scenarios of a transient study).  The solve then launches no kernel that
 * needs the whole device co-resident (the orthogonalization takes the
 * per-step kernels instead of the persistent launch); it requires the 2D
 * wavefront triangular solve or no preconditioner (else GG_EINVAL), whose
 * workgroups only wait on workgroups dispatched before them; for the same
 * reason the inner iteration's SpMV stays a launch of its own (without the
 * flag it runs inside the forward solve's launch on the GG_DIV_FMA 2D path;
 * environment GG_FUSE_SPMV=0 turns that off). */
#define GG_SOLVE_SHARED_DEVICE 0x1
/* gg_options.flags, the sharded solve (ggmres_dd.h) only: orthogonalize each
 * Arnoldi vector by classical Gram-Schmidt with one re-orthogonalization
 * (CGS2: h = V^T w, w -= V h, h2 = V^T w, w -= V h2, H[:, i] = h + h2) instead
 * of the reference's modified Gram-Schmidt (src/gmres.cu:2356-2359): three
 * all-gathers per inner iteration (h, h2, the norm) instead of i + 2.  A
 * different rounding (north_star's 1e-10 history tolerance); the default
 * stays MGS.  gg_solve refuses it (GG_EINVAL). */
#define GG_SOLVE_CGS2 0x2

typedef struct gg_result {
    int status;        /* GG_OK / GG_NOT_CONVERGED / error                        */
    int iters;         /* the reference's *max_iter output (src/gmres.cu:2174)    */
    int inner_iters;   /* Arnoldi iterations actually performed                   */
    int restarts;      /* restart cycles started                                  */
    double relres;     /* the reference's *tol output                             */
    double solve_ms;   /* device time of the solve phase (hipEvents)              */
} gg_result;

int gg_abi_version(void);
const char *gg_strerror(int status);
const char *gg_last_error(void);            /* detail of the last error on this thread */
int gg_device_count(int *count);

int gg_create(int device, gg_solver **out);
int gg_destroy(gg_solver *s);

int gg_set_matrix(gg_solver *s, int n, const int *row_ptr, const int *col_idx,
                  const double *val);

int gg_set_precond_none(gg_solver *s);
int gg_set_precond_ilu0(gg_solver *s);
/* the same ILU(0) with its numeric factorization on the GPU: leftILU
 * (src/leftILU.cu:27-336) factors level by level on the device; here one
 * dataflow launch processes every column once its sources are done.
 * Factors bit-identical to gg_set_precond_ilu0. */
int gg_set_precond_ilu0_device(gg_solver *s);
/* the device-factored matrix (L strict part divided by the pivots, U part) in
 * A's CSR order, before the 1e-9 drop / split; ms = device time (may be NULL) */
int gg_ilu0_device_values(gg_solver *s, double *val, double *ms);
int gg_set_precond_iluk(gg_solver *s, int level);
/* ILU(k) with ilukC's numeric elimination on the device (lofC's pattern and the
 * update lists built on the host, the reference's lofC is host code too); one
 * dataflow launch processes every row once the rows of its L part are done.
 * Factors bit-identical to gg_set_precond_iluk. GG_EZEROPIVOT as ilukC. */
int gg_set_precond_iluk_device(gg_solver *s, int level);
/* those device factors in the solver's forms (L unit lower, diagonal LAST; U
 * diagonal first); col/val arrays malloc'd by the library, release with
 * gg_host_free (ggmres_host.h); ms = device time (may be NULL) */
int gg_iluk_device_factors(gg_solver *s, int level, int *l_row_ptr, int **l_col_idx, double **l_val,
                           int *u_row_ptr, int **u_col_idx, double **u_val, double *ms);
/* L: unit lower (strict entries + unit diagonal LAST in each row; the diagonal is
 *    not applied, LUSolve_ignoreZero semantics); U: upper, diagonal first. */
int gg_set_precond_lu(gg_solver *s,
                      const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                      const int *u_row_ptr, const int *u_col_idx, const double *u_val);
/* ILU++/PG split preconditioner (MyILUPPfloat).  L: non-unit lower, diagonal LAST;
 * U: non-unit upper, diagonal FIRST; perm_row / perm_col as extracted at
 * src/mna_solve_gpu_gmres.cpp:396-474. */
int gg_set_precond_split(gg_solver *s,
                         const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                         const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                         const double *middle, const int *perm_row, const int *perm_col,
                         const double *lscale, const double *rscale);
/* A caller-supplied preconditioner: the reference's Preconditioner plug-in
 * (src/preconditioner.h:34-84), whose methods the engines call --
 * GMRES_GPU(..., Preconditioner&) (src/gmres.cu:2567-2732) DevPrecond, GMRESilu_GPU
 * (src/gmres.cu:2254-2446) DevPrecond_rhs / _left / _right / _starting_value.
 * The engine calls fn(ctx, op, in, out, n) with DEVICE arrays of n floats (the
 * reference's fp32 interface: the engine's fp64 vectors are rounded to float
 * for the call and the result promoted back), op = GG_APPLY_MINV (split = 0, the
 * left engine) or GG_APPLY_LEFT / RIGHT / START / RHS (split = 1, the split
 * engine).  fn runs on the calling host thread between the engine's kernels,
 * with the device synchronized before and after it (it may launch work on any
 * stream, or run on the host); it returns 0, or nonzero to abort the solve
 * (GG_EINVAL).  Natural order vector space, no triangular solve of the library's
 * own: the engine pays a host round trip per application. */
typedef int (*gg_precond_fn)(void *ctx, int op, const float *in, float *out, int n);
int gg_set_precond_user(gg_solver *s, int split, gg_precond_fn fn, void *ctx);
int gg_precond_kind(gg_solver *s);
/* Division in the non-unit triangular solves (the reference divides,
 * LUSolve_ignoreZero src/SpMV_compute.cpp:118-133, HostPrecond_left/right
 * src/preconditioner.cu:1094-1137):
 *   GG_DIV_EXACT (default)  x = RN(acc / d), bit-identical to the reference's
 *                           per-row arithmetic;
 *   GG_DIV_RCP              x = RN(acc * RN(1/d)) on the wavefront solves
 *                           (2D band / 3D tile): within about one ulp per row,
 *                           one multiply on the dependency chain instead of a
 *                           five-operation correctly rounded quotient, and one
 *                           streamed array fewer.  Tolerance parity (north_star
 *                           1e-10 on the residual history); the dataflow solve
 *                           of other sparsity keeps dividing;
 *   GG_DIV_FMA              on an unskewed 2D-grid wavefront (ILU(0) of a
 *                           5-point grid) every row is two fused multiply-adds,
 *                           in-line term first: x = fma(-c_l, x_l, fma(-c_i, x_i,
 *                           b)) for the unit L, and with c and b pre-scaled by
 *                           y = RN(1/d) (c' = RN(c*y), RN(b*y)) for U -- one
 *                           dependent FMA after the cross-lane move per step
 *                           instead of multiply, two subtractions and the
 *                           multiply by y.  A few ulps per row; tolerance parity
 *                           as GG_DIV_RCP, which the other wavefront solves fall
 *                           back to.
 * Applies to every later solve / apply of this solver. */
enum gg_div_mode { GG_DIV_EXACT = 0, GG_DIV_RCP = 1, GG_DIV_FMA = 2 };
int gg_set_division(gg_solver *s, int mode);
/* the division the last-set mode gives triangle `which` (0 = L / Ml, 1 = U /
 * Mr): GG_DIV_RCP only on a non-unit wavefront triangle whose 1/d are normal,
 * GG_DIV_FMA only on an unskewed 2D-grid wavefront triangle (the unit L, or a
 * non-unit U whose 1/d are normal) */
int gg_division_active(gg_solver *s, int which);
/* the kernel (rocprofv3 name) that runs triangle `which` (0 = L / Ml, 1 = U /
 * Mr) under the current division mode, into name[cap]; returns its length
 * ("" when the preconditioner has no triangles) */
int gg_trsv_kernel(gg_solver *s, int which, char *name, int cap);
/* the one-launch orthogonalization kernel of the last solve's inner
 * iterations (k_arnoldi_persist<J> / k_arnoldi_wide), "" when the per-step
 * kernels ran (or before the first solve); returns its length */
int gg_mgs_kernel(gg_solver *s, char *name, int cap);
/* the dependency chain of triangle `which` (0 = L / Ml, 1 = U / Mr): its
 * level count (the dataflow solve), or the wavefront's critical steps
 * (nx + skew (ny - 1) for a 2D band layout, nx + ny + nz - 2 for 3D) */
int gg_trsv_levels(gg_solver *s, int which);
/* 1 if the structured-grid wavefront triangular solve is active, else 0 */
int gg_uses_wavefront(gg_solver *s);
/* The solver's vector space, fixed by gg_set_precond_*: lay2nat[p] = the
 * natural row held at slot p (-1 = padding) for p < min(cap, Ppad); returns
 * Ppad (negative: error).  The 2D / 3D wavefront layouts, or off the
 * wavefront the natural order -- or, for the split engine's flow-kernel path,
 * an RCM order of the factors (GG_FLOW_RCM=0: natural).  Every reduction runs
 * in this order (tests: the order-matched oracle). */
long long gg_layout(gg_solver *s, long long *lay2nat, long long cap);
/* the block partials G of every dot in that space (the reduction grid the
 * solver actually uses, GG_WIDE_FORCE included) */
int gg_reduce_blocks(gg_solver *s, int *G);
/* the SpMV kernel the solver's matrix takes: 1 sliced ELL (k_spmv_sell: short,
 * evenly filled rows), 0 CSR-stream (k_spmv_stream); for y = A x a large
 * CSR-stream matrix with ascending rows may also run on column panels
 * (k_spmv_panel, gg_spmv_panels) */
int gg_spmv_sliced(gg_solver *s);
/* the number of column panels y = A x runs over (k_spmv_panel: x cut into
 * L2-sized panels, each row's terms added panel by panel into its running sum,
 * the CSR order), 0 when the matrix does not take them (GG_SPMV_PANEL) */
int gg_spmv_panels(gg_solver *s);
/* the column panels' launch form: > 0 = ONE launch of that many row blocks,
 * each walking its rows' segments panel by panel (k_spmv_rtile); 0 = one
 * launch per panel (k_spmv_panel, GG_SPMV_RTILE=0) or no panels */
int gg_spmv_rtile(gg_solver *s);

int gg_solve(gg_solver *s, const double *b, double *x, const gg_options *opt,
             gg_result *res);
int gg_solve_device(gg_solver *s, const double *d_b, double *d_x,
                    const gg_options *opt, gg_result *res);
/* fp32 device vectors (the reference's float* x / b, src/gmres.h:356-398): b
 * and x promoted to fp64 and x rounded back to fp32 ON the device (no host
 * round trip), natural order; otherwise as gg_solve_device */
int gg_solve_device_f32(gg_solver *s, const float *d_b, float *d_x, const gg_options *opt,
                        gg_result *res);
/* order-independent 64-bit fingerprints of `count` device buffers (bytes[i] a
 * multiple of 4): fp[i] = sum over the 32-bit words w_k of d_p[i] of
 * w_k * (2k + 1) modulo 2^64 -- one host round trip for all of them (the
 * engine ABI's check that a cached matrix was not changed in place) */
int gg_device_fingerprint(const void *const *d_p, const unsigned long long *bytes, int count,
                          unsigned long long *fp);
/* gg_set_matrix calls in this process (diagnostics: the engine ABI's setup
 * cache, compat/engine_abi.cpp) */
long long gg_set_matrix_count(void);
/* residual history of the last solve: [beta0/normb, |s[i+1]|/normb per inner
 * iteration, beta/normb after each restart ...] in event order.  Returns the
 * number of entries (may exceed cap; only cap are written). */
int gg_get_history(gg_solver *s, double *out, int cap);

/* single operators (host vectors, natural order) for parity tests */
int gg_spmv(gg_solver *s, const double *x, double *y);
int gg_precond_apply(gg_solver *s, int op, const double *in, double *out);

/* device-timed kernel measurements on the solver's stream (hipEvents).
 * gg_time_spmv: y = A x over nrot rotating copies of (x, y) so the Infinity
 * Cache cannot serve repeats when nrot * footprint > 256 MiB; avg_ms per launch.
 * nrot == 1 runs on the solver's own A and workspace (no copies, x = 1). */
int gg_time_spmv(gg_solver *s, int reps, int nrot, double *avg_ms);
/* average device time of one preconditioner application (L then U solve) */
int gg_time_precond(gg_solver *s, int reps, double *avg_ms);

/* In-solve kernel timing: every inner iteration brackets each selected kernel
 * family below with a hipEvent pair (timing-only events, no system fence) on
 * the solver's stream; totals accumulate over gg_solve* calls until
 * gg_profile_reset.  gg_profile_enable(s, kinds): kinds is a bit mask of
 * (1 << GG_PROF_*), GG_PROF_ALL for every family, 0 to switch timing off. */
enum gg_prof_kind {
    GG_PROF_SPMV = 0,      /* ww = A v_i                                  */
    GG_PROF_PRECOND = 1,   /* w = M^-1 ww (both triangular solves)        */
    GG_PROF_MGS = 2,       /* <w,v_0>, i+1 fused MGS steps, norm + Givens */
    GG_PROF_TRSV_L = 3,    /* the lower triangular solve alone (L / Ml)   */
    GG_PROF_TRSV_U = 4,    /* the upper triangular solve alone (U / Mr)   */
    GG_PROF_NKINDS = 5
};
#define GG_PROF_ALL ((1 << GG_PROF_NKINDS) - 1)
int gg_profile_enable(gg_solver *s, int kinds);
int gg_profile_reset(gg_solver *s);
int gg_profile_get(gg_solver *s, int kind, int *launches, double *total_ms);

/* bytes the solver moves per unit of work (algorithmic) */
double gg_bytes_spmv(gg_solver *s);
double gg_bytes_precond(gg_solver *s);
double gg_bytes_trsv(gg_solver *s, int which);   /* 0 = L / Ml, 1 = U / Mr */
/* what the triangular solve's kernel itself streams (the wavefront kernels read
 * no index arrays: less than gg_bytes_trsv's CSR formulation; otherwise equal) */
double gg_bytes_trsv_stream(gg_solver *s, int which);

/* Backward-Euler transient loop on one factorization: the step driver of
 * mna_solve_gpu_gmres (src/mna_solve_gpu_gmres.cpp:564-647) with PULSE sources
 * evaluated as gen_PULSEut_kernel (src/kernels.cu:223-245), entirely on the
 * device.  The matrix set by gg_set_matrix is A = G + C/h.  For it = 1..nsteps:
 *   u_k = PULSE_k(it * h)                      pulse: 7 doubles per source
 *                                              {vlo, vhi, td, tr, tf, tw, tp}
 *   w   = B u + (C/h) x                        B: source k adds +1 * u_k at row
 *                                              src_node[k]; cdiag = diag(C/h)
 *   x   = GMRES(A, w; warm start x)            opt as gg_solve
 *   port_out[j * (nsteps + 1) + it] = x[port[j]]   (column 0 = the initial x)
 * All arrays are host arrays; x (n doubles) is the initial state in and the
 * final state out, and stays in HBM between steps (only the right-hand side
 * assembly, the solves and the port capture run per step, all on the device).
 * *iters_total = sum of the per-step iteration counts (the reference's
 * iterTotal); returns GG_OK, or the status of the last non-converged step. */
int gg_transient(gg_solver *s, int nsteps, double h, const double *cdiag, int nsrc,
                 const int *src_node, const double *pulse, int nport, const int *port,
                 double *x, const gg_options *opt, double *port_out, int *iters_total);
/* Source kinds of gg_transient_src: the waveform generators of the reference's
 * GPU transient path (src/kernels.cu), evaluated at t = it * h for step it:
 *   GG_SRC_DC     data {value}                          gen_dcVt_kernel   (:73-85)
 *   GG_SRC_PULSE  data {vlo, vhi, td, tr, tf, tw, tp}   gen_PULSEut_kernel (:223-245)
 *   GG_SRC_PWL    data {t0, v0, t1, v1, ...}            gen_PWLut_kernel  (:146-176;
 *                 before t0 the value is v0, where the reference reads v[-1]) */
enum gg_src_kind { GG_SRC_DC = 0, GG_SRC_PULSE = 1, GG_SRC_PWL = 2 };
/* gg_transient with any mix of sources: source k at node src_node[k], kind
 * src_kind[k], parameters src_data[src_ptr[k] .. src_ptr[k+1]) */
int gg_transient_src(gg_solver *s, int nsteps, double h, const double *cdiag, int nsrc,
                     const int *src_node, const int *src_kind, const int *src_ptr, const double *src_data,
                     int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                     int *iters_total);
/* The step loop for a general MNA system (the wrapperGMRESforPG path,
 * src/wrapperGMRESforPG.cu:411-459, and the step driver's cs_dl_gaxpy forms,
 * src/mna_solve_gpu_gmres.cpp:585-591): the matrix set by gg_set_matrix is A
 * (G + C/h for the transient, G for a DC point); B is n x nsrc and R (= C/h,
 * capacitor stamps between nodes included) n x n, both CSR.  For step
 * j = 1..nsteps, with time index it = it0 + j - 1:
 *   u = sources(it * h)  (src_kind / src_ptr / src_data as gg_transient_src)
 *   w = B u + R x        (each row in ascending column order from 0.0; R may
 *                         be NULL: R = 0, a DC operating point)
 *   x = GMRES(A, w; warm start x)
 *   port_out[jp * (nsteps + 1) + j] = x[port[jp]]   (column 0 = the initial x)
 * Taps (gg_transient_set_taps) are tracked as in gg_transient. */
int gg_transient_mna(gg_solver *s, int it0, int nsteps, double h, const int *r_row_ptr, const int *r_col_idx,
                     const double *r_val, int nsrc, const int *b_row_ptr, const int *b_col_idx,
                     const double *b_val, const int *src_kind, const int *src_ptr, const double *src_data,
                     int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                     int *iters_total);
/* Tap-node statistics of the following gg_transient / gg_transient_src runs
 * (the step driver's ir_info block, src/mna_solve_gpu_gmres.cpp:285-292,
 * 633-645, 780-797): per tap node its maximum and minimum over the nsteps + 1
 * time points, its average (running sum in time order / (nsteps + 1)) and the
 * IR drop max - min.  set_taps(s, 0, NULL) turns it off; get_taps fills any
 * non-NULL array of ntap doubles from the last run. */
int gg_transient_set_taps(gg_solver *s, int ntap, const int *tap_node);
int gg_transient_get_taps(gg_solver *s, double *max_v, double *min_v, double *avg_v, double *ir);

/* ---- many right-hand sides (batch.hip; SURVEY.md 8(d) C5 "many-RHS") ----
 * nrhs independent systems A x_q = b_q on the solver's matrix and
 * preconditioner (the reference runs its step driver, src/mna_solve_gpu_gmres.
 * cpp:564-647, once per source scenario).  Scenario q's b / x at b + q * ldb /
 * x + q * ldx (natural order; x in = warm start, out = solution), res[q] its
 * result.  Each scenario runs exactly the single-RHS GMRES -- same iteration
 * count, history and solution bits as gg_solve_device on it alone -- while
 * every launch serves all of them: the SpMV reads A once for up to 8
 * scenarios, the wavefront triangular solves run every scenario's bands in one
 * launch (one dependency chain for all), each MGS launch reduces nrhs dots.
 * Batched when gg_batch_engine() = 1 (left ILU(0)/ILU(k)/LU factors of a 2D
 * grid on the unskewed wavefront); otherwise the scenarios are solved one
 * after the other with the same results.  Returns GG_OK when every scenario
 * converged, 1 when some did not, < 0 on error. */
int gg_solve_batch_device(gg_solver *s, int nrhs, const double *d_b, long long ldb, double *d_x, long long ldx,
                          const gg_options *opt, gg_result *res);
int gg_solve_batch(gg_solver *s, int nrhs, const double *b, long long ldb, double *x, long long ldx,
                   const gg_options *opt, gg_result *res);   /* host arrays */
/* 1 if batched launches serve gg_solve_batch*, 0 if scenario by scenario */
int gg_batch_engine(gg_solver *s);
/* scenario rhs's residual history of the last batched solve (as
 * gg_get_history): copies min(len, cap) entries, returns len */
long long gg_batch_history(gg_solver *s, int rhs, double *out, long long cap);
/* gg_transient_src for nrhs source scenarios at once, each its own source set,
 * all on the solver's A = G + C/h and cdiag: scenario q's sources are
 * k = src_off[q] .. src_off[q+1]-1 (node src_node[k], kind src_kind[k],
 * parameters src_data[src_ptr[k] .. src_ptr[k+1]), as gg_transient_src); x
 * holds nrhs states of n (in / out); port_out[(q * nport + j) * (nsteps + 1)
 * + it]; iters_total[q] per scenario.  Per step: every scenario's right-hand
 * side in one launch, then gg_solve_batch_device (warm start). */
int gg_transient_batch(gg_solver *s, int nrhs, int nsteps, double h, const double *cdiag, const int *src_off,
                       const int *src_node, const int *src_kind, const int *src_ptr, const double *src_data,
                       int nport, const int *port, double *x, const gg_options *opt, double *port_out,
                       int *iters_total);

/* Diagnostics: run one wavefront triangular solve (which: 0 = L / Ml, 1 = U / Mr)
 * on the current right-hand side and return, per band, the device real-time
 * clock (100 MHz) at the start of each batch (8 or 16 steps) plus one end stamp, then
 * core-cycle totals of four phases of the compute wave's batches (barrier wait,
 * batch top to first result, first to last result, last result to the next
 * barrier), the boundary wave's poll retries and the core cycles it spent
 * retrying, one spare slot, then the real-time stamps at which the writer wave
 * published each batch and at which the boundary wave saw each batch's
 * values: out[band * (3 * nbatch + 8) + k].  GG_ESTATE unless the wavefront path is active. */
int gg_trace_precond(gg_solver *s, int which, long long *out, long long cap, int *nbands,
                     int *nbatch);

#ifdef __cplusplus
}
#endif
#endif
