/*
 * oracle.c -- fp64 CPU restatement of the reference GPU-GMRES hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled with -ffp-contract=off
 * so every a*b+c is two roundings, as in the reference's scalar loops.
 * Reference citations are file:line in sheldonucr/GPU-GMRES.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* Equal(a, 0) with eps = 1e-9 (src/defs.h:45-47), evaluated with fabs. */
/* cpu_baseline_mt (bench.py): the same restatement built with -fopenmp
 * (liboracle_mt.so) runs the SpMV, BLAS-1 and update loops on every host core;
 * the triangular solves stay serial, as in the reference's host engine.  The
 * reductions then sum in another order: a timing baseline only, never a checker.
 * Without -fopenmp (liboracle.so, the checker) these expand to nothing. */
#ifdef _OPENMP
#include <omp.h>
int orc_threads(void) { return omp_get_max_threads(); }
#define ORC_PAR_FOR _Pragma("omp parallel for schedule(static)")
#define ORC_PAR_SUM(t) _Pragma("omp parallel for schedule(static) reduction(+:t)")
#else
int orc_threads(void) { return 1; }
#define ORC_PAR_FOR
#define ORC_PAR_SUM(t)
#endif

static int is_zero(double a) { return fabs(a) < 1e-9; }

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------ SpMV */
void orc_spmv(int n, const int *rp, const int *ci, const double *v,
              const double *x, double *y)
{
    /* computeSpMV (src/SpMV_compute.cpp:19-36): serial per-row sum in CSR order */
    ORC_PAR_FOR
    for (int i = 0; i < n; i++) {
        double t = 0.0;
        for (int j = rp[i]; j < rp[i + 1]; j++) t += v[j] * x[ci[j]];
        y[i] = t;
    }
}

void orc_residual(int n, const int *rp, const int *ci, const double *v,
                  const double *x, const double *b, double *r)
{
    /* sgemv(v, A, alpha=-1, x, beta=1, y=b) (src/gmres.cu:77-88) */
    double *t = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    orc_spmv(n, rp, ci, v, x, t);
    ORC_PAR_FOR
    for (int i = 0; i < n; i++) r[i] = -1.0 * t[i] + 1.0 * b[i];
    free(t);
}

/* ---------------------------------------------------------------- ILU(0) */
/* CSR -> CSC with rows ascending inside each column (csr2csc, src/leftILU.cu:371-417) */
static void csr_to_csc(int n, const int *rp, const int *ci, const double *v,
                       int *cp, int *ri, double *cv)
{
    int nnz = rp[n];
    int *cnt = (int *)calloc((size_t)n + 1, sizeof(int));
    for (int j = 0; j < nnz; j++) cnt[ci[j] + 1]++;
    cp[0] = 0;
    for (int c = 0; c < n; c++) cp[c + 1] = cp[c] + cnt[c + 1];
    int *pos = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int c = 0; c < n; c++) pos[c] = cp[c];
    for (int r = 0; r < n; r++)
        for (int j = rp[r]; j < rp[r + 1]; j++) {
            int c = ci[j];
            ri[pos[c]] = r;
            cv[pos[c]] = v[j];
            pos[c]++;
        }
    free(pos);
    free(cnt);
}

/* liSearchLowerBound (src/leftILU.cu:831-840) */
static int lower_bound_lin(int target, int lpos, int upos, const int *a)
{
    for (int i = lpos; i < upos; i++)
        if (a[i] >= target) return i;
    return upos;
}

/* cpuSequentialTriSolve body for one column (src/leftILU.cu:774-821) */
static void ilu0_column(int tgt, const int *cp, const int *ri, double *cv)
{
    int lb = cp[tgt], ub = cp[tgt + 1];
    double u_diag = 0.0;
    for (int k = lb; k < ub - 1; k++) {
        int cur_row = ri[k];
        if (cur_row > tgt) break;
        if (cur_row == tgt) { u_diag = cv[k]; break; }
        int left_lb = cp[cur_row], left_ub = cp[cur_row + 1];
        for (int p = k + 1; p < ub; p++) {
            int r2 = ri[p];
            int q = lower_bound_lin(r2, left_lb, left_ub, ri);
            if (q < left_ub && ri[q] == r2) cv[p] -= cv[q] * cv[k];
        }
    }
    for (int k = lb; k < ub; k++) {
        if (ri[k] <= tgt) continue;
        if (!is_zero(u_diag)) cv[k] /= u_diag;
        else cv[k] = 0.0;
    }
}

/* splitLU_csr (src/leftILU.cu:481-541): drop |v|<1e-9, L gets a unit diag LAST */
static void split_lu(int n, const int *rp, const int *ci, const double *v,
                     int *l_rp, int **l_ci, double **l_v,
                     int *u_rp, int **u_ci, double **u_v)
{
    l_rp[0] = 0; u_rp[0] = 0;
    for (int r = 0; r < n; r++) {
        int nl = 0, nu = 0;
        for (int j = rp[r]; j < rp[r + 1]; j++) {
            if (is_zero(v[j])) continue;
            if (ci[j] < r) nl++; else nu++;
        }
        l_rp[r + 1] = l_rp[r] + nl + 1;
        u_rp[r + 1] = u_rp[r] + nu;
    }
    *l_ci = (int *)malloc((size_t)(l_rp[n] > 0 ? l_rp[n] : 1) * sizeof(int));
    *l_v = (double *)malloc((size_t)(l_rp[n] > 0 ? l_rp[n] : 1) * sizeof(double));
    *u_ci = (int *)malloc((size_t)(u_rp[n] > 0 ? u_rp[n] : 1) * sizeof(int));
    *u_v = (double *)malloc((size_t)(u_rp[n] > 0 ? u_rp[n] : 1) * sizeof(double));
    for (int r = 0; r < n; r++) {
        int pl = l_rp[r], pu = u_rp[r];
        for (int j = rp[r]; j < rp[r + 1]; j++) {
            if (is_zero(v[j])) continue;
            if (ci[j] < r) { (*l_ci)[pl] = ci[j]; (*l_v)[pl] = v[j]; pl++; }
            else { (*u_ci)[pu] = ci[j]; (*u_v)[pu] = v[j]; pu++; }
        }
        (*l_ci)[pl] = r; (*l_v)[pl] = 1.0;
    }
}

/* leftILU's factorization up to (excluding) the split: the factored matrix in
 * CSR form (crp/cci/cvv, malloc'd; same pattern and order as a sorted A) */
static void ilu0_factor_csr(int n, const int *rp, const int *ci, const double *v,
                            int **crp_out, int **cci_out, double **cvv_out)
{
    int nnz = rp[n];
    size_t cap = (size_t)(nnz > 0 ? nnz : 1);
    /* generateLevel (src/leftILU.cu:339-368) on the original values */
    int *level = (int *)calloc((size_t)n + 1, sizeof(int));
    int maxlev = 0;
    for (int r = 0; r < n; r++)
        for (int j = rp[r]; j < rp[r + 1]; j++)
            if (!is_zero(v[j]) && ci[j] > r) {
                int c = ci[j];
                if (level[c] < level[r] + 1) level[c] = level[r] + 1;
            }
    for (int r = 0; r < n; r++) if (level[r] > maxlev) maxlev = level[r];
    /* egraph: columns bucketed by level, ascending index inside a level (:41-49) */
    int *lcnt = (int *)calloc((size_t)maxlev + 2, sizeof(int));
    for (int r = 0; r < n; r++) lcnt[level[r] + 1]++;
    for (int l = 0; l <= maxlev; l++) lcnt[l + 1] += lcnt[l];
    int *order = (int *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int r = 0; r < n; r++) order[lcnt[level[r]]++] = r;

    int *cp = (int *)malloc(((size_t)n + 1) * sizeof(int));
    int *ri = (int *)malloc(cap * sizeof(int));
    double *cv = (double *)malloc(cap * sizeof(double));
    csr_to_csc(n, rp, ci, v, cp, ri, cv);
    /* the reference runs its GPU kernel sparseTriSolve_V2 on levels >= 32 nodes;
     * that kernel races, so every column follows
     * the CPU kernel here, in the same level order */
    for (int k = 0; k < n; k++) ilu0_column(order[k], cp, ri, cv);

    /* csr2csc(csc) back to CSR (src/leftILU.cu:297), then split (:298) */
    int *crp = (int *)malloc(((size_t)n + 1) * sizeof(int));
    int *cci = (int *)malloc(cap * sizeof(int));
    double *cvv = (double *)malloc(cap * sizeof(double));
    csr_to_csc(n, cp, ri, cv, crp, cci, cvv); /* transpose of CSC == CSR */
    *crp_out = crp; *cci_out = cci; *cvv_out = cvv;
    free(cp); free(ri); free(cv);
    free(order); free(lcnt); free(level);
}

int orc_ilu0(int n, const int *rp, const int *ci, const double *v,
             int *l_rp, int **l_ci, double **l_v,
             int *u_rp, int **u_ci, double **u_v)
{
    int *crp, *cci;
    double *cvv;
    ilu0_factor_csr(n, rp, ci, v, &crp, &cci, &cvv);
    split_lu(n, crp, cci, cvv, l_rp, l_ci, l_v, u_rp, u_ci, u_v);
    free(crp); free(cci); free(cvv);
    return 0;
}

int orc_ilu0_values(int n, const int *rp, const int *ci, const double *v, double *out)
{
    int *crp, *cci;
    double *cvv;
    ilu0_factor_csr(n, rp, ci, v, &crp, &cci, &cvv);
    memcpy(out, cvv, (size_t)rp[n] * sizeof(double));
    free(crp); free(cci); free(cvv);
    return 0;
}

/* ---------------------------------------------------------------- ILU(k) */
static int cmp_int_pair(const void *a, const void *b)
{
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

int orc_iluk(int lofM, int n, const int *rp, const int *ci, const double *v,
             int *l_rp, int **l_ci, double **l_v,
             int *u_rp, int **u_ci, double **u_v)
{
    /* symbolic: lofC (src/iluk.cpp:192-334) */
    int **Lja = (int **)calloc((size_t)n + 1, sizeof(int *));
    int **Uja = (int **)calloc((size_t)n + 1, sizeof(int *));
    int **ulvl = (int **)calloc((size_t)n + 1, sizeof(int *));
    int *Lnz = (int *)calloc((size_t)n + 1, sizeof(int));
    int *Unz = (int *)calloc((size_t)n + 1, sizeof(int));
    int *levls = (int *)malloc(((size_t)n + 1) * sizeof(int));
    int *jbuf = (int *)malloc(((size_t)n + 1) * sizeof(int));
    int *iw = (int *)malloc(((size_t)n + 1) * sizeof(int));
    for (int j = 0; j < n; j++) iw[j] = -1;
    for (int i = 0; i < n; i++) {
        int incl = 0, incu = i;
        for (int j = rp[i]; j < rp[i + 1]; j++) {
            int col = ci[j];
            if (col < i) { jbuf[incl] = col; levls[incl] = 0; iw[col] = incl++; }
            else if (col > i) { jbuf[incu] = col; levls[incu] = 0; iw[col] = incu++; }
        }
        int jpiv = -1;
        while (++jpiv < incl) {
            int k = jbuf[jpiv], kmin = k, jmin = jpiv;
            for (int j = jpiv + 1; j < incl; j++)
                if (jbuf[j] < kmin) { kmin = jbuf[j]; jmin = j; }
            if (jmin != jpiv) {  /* select leftmost pivot (:263-281) */
                jbuf[jpiv] = kmin; jbuf[jmin] = k;
                iw[kmin] = jpiv; iw[k] = jmin;
                int t = levls[jpiv]; levls[jpiv] = levls[jmin]; levls[jmin] = t;
                k = kmin;
            }
            for (int j = 0; j < Unz[k]; j++) {
                int col = Uja[k][j];
                int it = ulvl[k][j] + levls[jpiv] + 1;
                if (it > lofM) continue;
                int ip = iw[col];
                if (ip == -1) {
                    if (col < i) { jbuf[incl] = col; levls[incl] = it; iw[col] = incl++; }
                    else if (col > i) { jbuf[incu] = col; levls[incu] = it; iw[col] = incu++; }
                } else if (it < levls[ip]) {
                    levls[ip] = it;
                }
            }
        }
        for (int j = 0; j < incl; j++) iw[jbuf[j]] = -1;
        for (int j = i; j < incu; j++) iw[jbuf[j]] = -1;
        Lnz[i] = incl;
        Lja[i] = (int *)malloc((size_t)(incl > 0 ? incl : 1) * sizeof(int));
        memcpy(Lja[i], jbuf, sizeof(int) * (size_t)incl);
        int ku = incu - i;
        Unz[i] = ku;
        Uja[i] = (int *)malloc((size_t)(ku > 0 ? ku : 1) * sizeof(int));
        ulvl[i] = (int *)malloc((size_t)(ku > 0 ? ku : 1) * sizeof(int));
        memcpy(Uja[i], jbuf + i, sizeof(int) * (size_t)ku);
        memcpy(ulvl[i], levls + i, sizeof(int) * (size_t)ku);
    }
    /* numeric: ilukC (src/iluk.cpp:56-190), diagonal kept inverted in D */
    double **Lma = (double **)calloc((size_t)n + 1, sizeof(double *));
    double **Uma = (double **)calloc((size_t)n + 1, sizeof(double *));
    double *D = (double *)malloc(((size_t)n + 1) * sizeof(double));
    double *Draw = (double *)malloc(((size_t)n + 1) * sizeof(double));
    int *jw = iw;
    int ierr = 0;
    for (int j = 0; j < n; j++) jw[j] = -1;
    for (int i = 0; i < n && !ierr; i++) {
        Lma[i] = (double *)malloc((size_t)(Lnz[i] > 0 ? Lnz[i] : 1) * sizeof(double));
        Uma[i] = (double *)malloc((size_t)(Unz[i] > 0 ? Unz[i] : 1) * sizeof(double));
        for (int j = 0; j < Lnz[i]; j++) { jw[Lja[i][j]] = j; Lma[i][j] = 0.0; }
        jw[i] = i;
        D[i] = 0.0;
        for (int j = 0; j < Unz[i]; j++) { jw[Uja[i][j]] = j; Uma[i][j] = 0.0; }
        for (int j = rp[i]; j < rp[i + 1]; j++) {
            int col = ci[j], jpos = jw[col];
            if (col < i) Lma[i][jpos] = v[j];
            else if (col == i) D[i] = v[j];
            else Uma[i][jpos] = v[j];
        }
        for (int j = 0; j < Lnz[i]; j++) {
            int jrow = Lja[i][j];
            Lma[i][j] *= D[jrow];
            for (int k = 0; k < Unz[jrow]; k++) {
                int col = Uja[jrow][k], jpos = jw[col];
                if (jpos == -1) continue;
                if (col < i) Lma[i][jpos] -= Lma[i][j] * Uma[jrow][k];
                else if (col == i) D[i] -= Lma[i][j] * Uma[jrow][k];
                else Uma[i][jpos] -= Lma[i][j] * Uma[jrow][k];
            }
        }
        for (int j = 0; j < Lnz[i]; j++) jw[Lja[i][j]] = -1;
        jw[i] = -1;
        for (int j = 0; j < Unz[i]; j++) jw[Uja[i][j]] = -1;
        if (D[i] == 0.0) { ierr = -2; break; }
        Draw[i] = D[i];
        D[i] = 1.0 / D[i];
    }
    if (!ierr) {
        /* emit: L strict (ascending, as lofC leaves it) + unit diag last;
         * U: diag (un-inverted) first, strict upper sorted ascending */
        l_rp[0] = 0; u_rp[0] = 0;
        for (int i = 0; i < n; i++) {
            l_rp[i + 1] = l_rp[i] + Lnz[i] + 1;
            u_rp[i + 1] = u_rp[i] + Unz[i] + 1;
        }
        *l_ci = (int *)malloc((size_t)l_rp[n] * sizeof(int) + 4);
        *l_v = (double *)malloc((size_t)l_rp[n] * sizeof(double) + 8);
        *u_ci = (int *)malloc((size_t)u_rp[n] * sizeof(int) + 4);
        *u_v = (double *)malloc((size_t)u_rp[n] * sizeof(double) + 8);
        int *pairs = (int *)malloc(((size_t)n + 1) * 2 * sizeof(int));
        for (int i = 0; i < n; i++) {
            int p = l_rp[i];
            for (int j = 0; j < Lnz[i]; j++) { (*l_ci)[p] = Lja[i][j]; (*l_v)[p] = Lma[i][j]; p++; }
            (*l_ci)[p] = i; (*l_v)[p] = 1.0;
            p = u_rp[i];
            (*u_ci)[p] = i; (*u_v)[p] = Draw[i]; p++;
            for (int j = 0; j < Unz[i]; j++) { pairs[2 * j] = Uja[i][j]; pairs[2 * j + 1] = j; }
            qsort(pairs, (size_t)Unz[i], 2 * sizeof(int), cmp_int_pair);
            for (int j = 0; j < Unz[i]; j++) {
                (*u_ci)[p] = pairs[2 * j]; (*u_v)[p] = Uma[i][pairs[2 * j + 1]]; p++;
            }
        }
        free(pairs);
    }
    for (int i = 0; i < n; i++) {
        free(Lja[i]); free(Uja[i]); free(ulvl[i]); free(Lma[i]); free(Uma[i]);
    }
    free(Lja); free(Uja); free(ulvl); free(Lma); free(Uma);
    free(Lnz); free(Unz); free(levls); free(jbuf); free(iw); free(D); free(Draw);
    return ierr;
}

/* ------------------------------------------------------- triangular solve */
/* Division mode of the non-unit triangles (the device's gg_set_division):
 * 0 = x / d as the reference; 1 = x * (1.0 / d), the device's WD_MUL
 * (x = RN(acc * RN(1/d))), per triangle (L = the lower / Ml one, U = the upper
 * / Mr one).  Only for order-matched checks of GG_DIV_RCP solves.
 * 2 = the device's GG_DIV_FMA rows (kernels.hip WD_UFMA / WD_SFMA; orc_lusolve
 * and the split engine's two solves): with y = RN(1/d) (y = 1 for the unit L),
 * acc = RN(b*y) (b for the unit L), then for the off-diagonal terms nearest
 * first (|i - col| ascending) acc = fma(-RN(c*y), x[col], acc) (c for the unit L). */
static int g_mul_l = 0, g_mul_u = 0;
void orc_set_div_mode(int mul_l, int mul_u)
{
    g_mul_l = mul_l < 0 ? 0 : mul_l > 2 ? 2 : mul_l;
    g_mul_u = mul_u < 0 ? 0 : mul_u > 2 ? 2 : mul_u;
}
/* GG_DIV_FMA on a bordered grid (the device's Wave2D::bnt, split engine): in
 * the Ml rows below the first `tail` rows the terms of columns < tail (the
 * tail, pads and branch currents) come first, in canonical order, then the
 * rest nearest first -- the tail's contribution is formed before the mesh's
 * wavefront starts the row.  0 = no tail (every row nearest first). */
static int g_fma_tail = 0;
void orc_set_fma_tail(int tail) { g_fma_tail = tail > 0 ? tail : 0; }
static double divide(double a, double d, int mul) { return mul ? a * (1.0 / d) : a / d; }

void orc_lusolve(int n, const int *l_rp, const int *l_ci, const double *l_v,
                 const int *u_rp, const int *u_ci, const double *u_v,
                 const double *y, double *x)
{
    /* LUSolve_ignoreZero (src/SpMV_compute.cpp:92-136).  The L diagonal is
     * never applied (the reference divides the scratch x, :112), i.e. unit L. */
    double *w = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    memcpy(w, y, (size_t)n * sizeof(double));
    for (int i = 0; i < n; i++) {
        if (g_mul_l == 2) {         /* GG_DIV_FMA: nearest term first, fused */
            int j = l_rp[i];
            while (j < l_rp[i + 1] && l_ci[j] < i) j++;
            double acc = w[i];
            for (j--; j >= l_rp[i]; j--) acc = fma(-l_v[j], w[l_ci[j]], acc);
            w[i] = acc;
            continue;
        }
        for (int j = l_rp[i]; j < l_rp[i + 1]; j++) {
            if (l_ci[j] >= i) break;
            w[i] -= l_v[j] * w[l_ci[j]];
        }
    }
    memcpy(x, w, (size_t)n * sizeof(double));
    for (int i = n - 1; i >= 0; i--) {
        if (g_mul_u == 2) {         /* GG_DIV_FMA: pre-scaled by RN(1/d), nearest term first */
            int j = u_rp[i];
            while (j < u_rp[i + 1] && u_ci[j] < i) j++;
            double yd = 1.0;
            if (j < u_rp[i + 1] && u_ci[j] == i && !is_zero(u_v[j])) yd = 1.0 / u_v[j];
            if (j < u_rp[i + 1] && u_ci[j] == i) j++;
            double acc = x[i] * yd;
            for (; j < u_rp[i + 1]; j++) acc = fma(-(u_v[j] * yd), x[u_ci[j]], acc);
            x[i] = acc;
            continue;
        }
        int lb = u_rp[i], j = u_rp[i + 1] - 1;
        for (; j >= lb; j--) {
            if (u_ci[j] <= i) break;
            x[i] -= u_v[j] * x[u_ci[j]];
        }
        if (j >= lb && u_ci[j] == i && !is_zero(u_v[j])) x[i] = divide(x[i], u_v[j], g_mul_u);
    }
    free(w);
}

/* ---------------------------------------------- split (PG) preconditioner */
void orc_split_left(const orc_split_t *p, const double *in, double *out)
{
    /* MyILUPP::HostPrecond_left (src/preconditioner.cu:1094-1114) */
    int n = p->n;
    double *t = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int i = 0; i < n; i++) t[i] = in[i] / p->lscale[i];
    for (int i = 0; i < n; i++) out[i] = t[p->perm_row[i]];
    for (int i = 0; i < n; i++) {
        int lb = p->l_rp[i], ub = p->l_rp[i + 1];
        if (g_mul_l == 2) {         /* GG_DIV_FMA: pre-scaled, nearest term first */
            double yd = 1.0 / p->l_v[ub - 1], acc = out[i] * yd;
            int j0 = lb;            /* (a bordered grid's mesh row: its tail terms first) */
            if (i >= g_fma_tail)
                for (; j0 < ub - 1 && p->l_ci[j0] < g_fma_tail; j0++)
                    acc = fma(-(p->l_v[j0] * yd), out[p->l_ci[j0]], acc);
            for (int j = ub - 2; j >= j0; j--) acc = fma(-(p->l_v[j] * yd), out[p->l_ci[j]], acc);
            out[i] = acc;
            continue;
        }
        for (int j = lb; j < ub - 1; j++) out[i] -= p->l_v[j] * out[p->l_ci[j]];
        out[i] = divide(out[i], p->l_v[ub - 1], g_mul_l);
    }
    free(t);
}

void orc_split_right(const orc_split_t *p, const double *in, double *out)
{
    /* MyILUPP::HostPrecond_right (src/preconditioner.cu:1117-1137) */
    int n = p->n;
    double *t = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int i = 0; i < n; i++) t[i] = in[i] * p->middle[i];
    for (int i = n - 1; i >= 0; i--) {
        int lb = p->u_rp[i], ub = p->u_rp[i + 1];
        if (g_mul_u == 2) {         /* GG_DIV_FMA: pre-scaled, nearest term first */
            double yd = 1.0 / p->u_v[lb], acc = t[i] * yd;
            for (int j = lb + 1; j < ub; j++) acc = fma(-(p->u_v[j] * yd), t[p->u_ci[j]], acc);
            t[i] = acc;
            continue;
        }
        for (int j = lb + 1; j < ub; j++) t[i] -= p->u_v[j] * t[p->u_ci[j]];
        t[i] = divide(t[i], p->u_v[lb], g_mul_u);
    }
    for (int i = 0; i < n; i++) out[i] = t[p->perm_col[i]] / p->rscale[i];
    free(t);
}

void orc_split_start(const orc_split_t *p, const double *in, double *out)
{
    /* MyILUPP::HostPrecond_starting_value (src/preconditioner.cu:1074-1091) */
    int n = p->n;
    double *t = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    double *z = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int i = 0; i < n; i++) t[i] = in[i] * p->rscale[i];
    for (int i = 0; i < n; i++) z[p->perm_col[i]] = t[i];
    for (int i = 0; i < n; i++) {
        double s = 0.0;
        for (int j = p->u_rp[i]; j < p->u_rp[i + 1]; j++) s += p->u_v[j] * z[p->u_ci[j]];
        t[i] = s;
    }
    for (int i = 0; i < n; i++) out[i] = t[i] / p->middle[i];
    free(z);
    free(t);
}

/* ---------------------------------------------------------------- Givens */
void orc_apply_rot(double *dx, double *dy, double cs, double sn)
{
    /* ApplyPlaneRotation (src/gmres.cu:192-197) */
    double temp = cs * (*dx) + sn * (*dy);
    *dy = -sn * (*dx) + cs * (*dy);
    *dx = temp;
}

void orc_gen_rot(double dx, double dy, double *cs, double *sn)
{
    /* GeneratePlaneRotation (src/gmres.cu:200-216): 1/sqrt(1+t^2), not hypot */
    if (dy == 0.0) { *cs = 1.0; *sn = 0.0; }
    else if (fabs(dy) > fabs(dx)) {
        double temp = dx / dy;
        *sn = 1.0 / sqrt(1.0 + temp * temp);
        *cs = temp * (*sn);
    } else {
        double temp = dy / dx;
        *cs = 1.0 / sqrt(1.0 + temp * temp);
        *sn = temp * (*cs);
    }
}

/* ------------------------------------------------------------ BLAS-1 */
/* Summation order of dot products / norms.  The reference's CPU engine sums
 * serially (src/gmres.cu:60-74); its GPU engine calls cublasSdot/Snrm2, a
 * parallel tree of unspecified order.  Mode "blocked" restates one concrete
 * tree -- the device kernels' (DESIGN.md "Reduction order") -- so a solve can
 * be compared bit-for-bit: vectors laid out by lay2nat over ppad slots
 * (-1 = padding zero), G blocks of 256 threads, each thread summing its
 * grid-stride double2 units, 64-lane xor butterflies, (w0+w1)+(w2+w3). */
static int g_blocked = 0;
static long long g_ppad = 0;
static int g_G = 1;
static const long long *g_lay2nat = NULL;
/* the sharded solve (gpu-gmres_amd/csrc/dd.hip): nseg shards, shard s summing
 * its own dot range of seglen[s] slots (lay2nat segments concatenated) into G
 * block partials; the nseg*G partials (shard-major) are then summed as above */
static int g_nseg = 1;
static const long long *g_seglen = NULL;

void orc_set_dot_order(int blocked, long long ppad, int G, const long long *lay2nat)
{
    g_blocked = blocked;
    g_ppad = ppad;
    g_G = G > 0 ? G : 1;
    g_lay2nat = lay2nat;
    g_nseg = 1;
    g_seglen = NULL;
}

void orc_set_dot_order_shards(int nseg, const long long *seglen, int G, const long long *lay2nat)
{
    g_blocked = nseg > 0;
    g_nseg = nseg > 0 ? nseg : 1;
    g_seglen = seglen;
    g_G = G > 0 ? G : 1;
    g_lay2nat = lay2nat;
    g_ppad = 0;
}

static double block_sum256(double *v)
{
    double t[256];
    for (int w = 0; w < 4; w++)
        for (int o = 32; o > 0; o >>= 1) {
            for (int l = 0; l < 64; l++) t[w * 64 + l] = v[w * 64 + l] + v[w * 64 + (l ^ o)];
            for (int l = 0; l < 64; l++) v[w * 64 + l] = t[w * 64 + l];
        }
    return (v[0] + v[64]) + (v[128] + v[192]);
}

static double dot_blocked(const double *x, const double *y)
{
    const int nparts = g_nseg * g_G;
    double *part = (double *)malloc((size_t)nparts * sizeof(double));
    double v[256];
    long long base = 0;
    for (int sg = 0; sg < g_nseg; sg++) {
        const long long len = g_seglen ? g_seglen[sg] : g_ppad;
        const long long units = len / 2;
        const long long *l2n = g_lay2nat + base;
        for (int blk = 0; blk < g_G; blk++) {
            for (int t = 0; t < 256; t++) {
                double acc = 0.0;
                for (long long u = (long long)blk * 256 + t; u < units; u += (long long)g_G * 256) {
                    long long p0 = l2n[2 * u], p1 = l2n[2 * u + 1];
                    double a0 = p0 >= 0 ? x[p0] : 0.0, b0 = p0 >= 0 ? y[p0] : 0.0;
                    double a1 = p1 >= 0 ? x[p1] : 0.0, b1 = p1 >= 0 ? y[p1] : 0.0;
                    acc += a0 * b0;
                    acc += a1 * b1;
                }
                v[t] = acc;
            }
            part[sg * g_G + blk] = block_sum256(v);
        }
        base += len;
    }
    for (int t = 0; t < 256; t++) {
        double acc = 0.0;
        for (int k = t; k < nparts; k += 256) acc += part[k];
        v[t] = acc;
    }
    double r = block_sum256(v);
    free(part);
    return r;
}

static double dot(const double *x, const double *y, int n)
{
    if (g_blocked) return dot_blocked(x, y);
    double t = 0.0;                 /* dot (src/gmres.cu:68-74) */
    ORC_PAR_SUM(t)
    for (int i = 0; i < n; i++) t += x[i] * y[i];
    return t;
}
static double norm2(const double *v, int n)
{
    if (g_blocked) return sqrt(dot_blocked(v, v));
    double t = 0.0;                 /* norm2 (src/gmres.cu:60-66) */
    ORC_PAR_SUM(t)
    for (int i = 0; i < n; i++) t += v[i] * v[i];
    return sqrt(t);
}

/* Orthogonalization: 0 = modified Gram-Schmidt as the reference
 * (src/gmres.cu:638-641, 2356-2359); 1 = CGS2, the sharded solve's
 * GG_SOLVE_CGS2 (csrc/kernels.hip k_multidot / k_cgs_reduce / k_cgs_update):
 * h_k = <w, v_k> for every k from the same w, then per element
 * w = (-h_k) v_k + w for k ascending, the same again with h2, H = h + h2. */
static int g_orth = 0;
void orc_set_orth(int cgs2) { g_orth = cgs2 != 0; }

/* Update (src/gmres.cu:93-116): y = H(0:k,0:k)^-1 s; x += V y */
static void update(double *x, int k, const double *H, int m, const double *s,
                   const double *V, int n)
{
    double *y = (double *)malloc((size_t)(k + 1) * sizeof(double));
    for (int i = 0; i <= k; i++) y[i] = s[i];
    for (int i = k; i >= 0; i--) {
        y[i] /= H[i + i * (m + 1)];
        for (int j = i - 1; j >= 0; j--) y[j] -= H[j + i * (m + 1)] * y[i];
    }
    for (int j = 0; j <= k; j++) {
        ORC_PAR_FOR
        for (int i = 0; i < n; i++) x[i] += V[(size_t)j * n + i] * y[j];
    }
    free(y);
}

typedef struct {
    double *h; int cap; int len;
} hist_t;
static void hist_push(hist_t *h, double v)
{
    if (h->h && h->len < h->cap) h->h[h->len] = v;
    h->len++;
}

/* Operator abstraction so GMRES_leftILU0 and GMRESilu share one restated loop.
 * kind 0 = left ILU (M^-1 = (LU)^-1), kind 1 = split PG. */
typedef struct {
    int kind;
    int n;
    const int *rp, *ci; const double *v;
    const int *l_rp, *l_ci; const double *l_v;
    const int *u_rp, *u_ci; const double *u_v;
    const orc_split_t *sp;
} op_t;

static int gmres_core(const op_t *op, const double *b, double *x, int m,
                      int *max_iter, double *tol, double *hist, int hist_cap,
                      int *hist_len, int *inner_iters)
{
    int n = op->n;
    size_t nn = (size_t)(n > 0 ? n : 1);
    double resid;
    int i, j = 1, k;
    int done_iters = 0;
    double *s = (double *)calloc((size_t)m + 1, sizeof(double));
    double *cs = (double *)calloc((size_t)m + 1, sizeof(double));
    double *sn = (double *)calloc((size_t)m + 1, sizeof(double));
    double *w = (double *)malloc(nn * sizeof(double));
    double *ww = (double *)malloc(nn * sizeof(double));
    double *r = (double *)malloc(nn * sizeof(double));
    double *rr = (double *)malloc(nn * sizeof(double));
    double *bb = (double *)malloc(nn * sizeof(double));
    double *H = (double *)calloc((size_t)(m + 1) * (size_t)m, sizeof(double));
    double *V = (double *)malloc((size_t)(m + 1) * nn * sizeof(double));
    double *y = (double *)calloc(nn, sizeof(double));   /* split: Mr^-1 x */
    double *s_cgs = (double *)calloc((size_t)m + 1, sizeof(double));
    double *acc = x;                                     /* left: update x directly */
    hist_t hs = {hist, hist_cap, 0};
    int ret = 1;

    /* normb = ||M b||  (left: :593-594 ; split: HostPrecond_rhs :2096-2098) */
    if (op->kind == 0)
        orc_lusolve(n, op->l_rp, op->l_ci, op->l_v, op->u_rp, op->u_ci, op->u_v, b, bb);
    else
        orc_split_left(op->sp, b, bb);
    double normb = norm2(bb, n);
    if (normb == 0.0) normb = 1.0;

    if (op->kind == 1) {
        orc_split_start(op->sp, x, y);   /* :2102 */
        acc = y;
    }
    orc_residual(n, op->rp, op->ci, op->v, x, b, rr);
    if (op->kind == 0)
        orc_lusolve(n, op->l_rp, op->l_ci, op->l_v, op->u_rp, op->u_ci, op->u_v, rr, r);
    else
        orc_split_left(op->sp, rr, r);
    double beta = norm2(r, n);
    resid = beta / normb;
    hist_push(&hs, resid);
    if (resid <= *tol) {                 /* note "<=" (:608 / :2112) */
        *tol = resid;
        *max_iter = 0;
        ret = 0;
        goto out;
    }

    while (j <= *max_iter) {
        double inv = 1.0 / beta;
        ORC_PAR_FOR
        for (int t = 0; t < n; t++) V[t] = inv * r[t];
        for (int t = 0; t <= m; t++) s[t] = 0.0;
        s[0] = beta;
        for (i = 0; i < m && j <= *max_iter; i++, j++) {
            double *vi = V + (size_t)i * nn;
            if (op->kind == 0) {
                orc_spmv(n, op->rp, op->ci, op->v, vi, ww);              /* :635 */
                orc_lusolve(n, op->l_rp, op->l_ci, op->l_v, op->u_rp, op->u_ci,
                            op->u_v, ww, w);                           /* :636 */
            } else {
                orc_split_right(op->sp, vi, w);                        /* :2143 */
                orc_spmv(n, op->rp, op->ci, op->v, w, ww);             /* :2144 */
                orc_split_left(op->sp, ww, w);                         /* :2145 */
            }
            if (g_orth == 1) {                                         /* CGS2 (GG_SOLVE_CGS2) */
                for (int pass = 0; pass < 2; pass++) {
                    for (k = 0; k <= i; k++) {
                        const double h = dot(w, V + (size_t)k * nn, n);
                        s_cgs[k] = h;
                        H[k + i * (m + 1)] = pass ? H[k + i * (m + 1)] + h : h;
                    }
                    for (int t = 0; t < n; t++) {
                        double wt = w[t];
                        for (k = 0; k <= i; k++) wt = (-s_cgs[k]) * V[(size_t)k * nn + t] + wt;
                        w[t] = wt;
                    }
                }
            } else {
                for (k = 0; k <= i; k++) {                             /* MGS :638-641 */
                    const double *vk = V + (size_t)k * nn;
                    double h = dot(w, vk, n);
                    H[k + i * (m + 1)] = h;
                    double a = -h;
                    ORC_PAR_FOR
                    for (int t = 0; t < n; t++) w[t] = a * vk[t] + w[t];
                }
            }
            double hn = norm2(w, n);
            H[(i + 1) + i * (m + 1)] = hn;
            /* v_{i+1} = w * (1/H(i+1,i)) (:645); lucky breakdown guarded */
            double *vn = V + (size_t)(i + 1) * nn;
            if (hn != 0.0) {
                double hinv = 1.0 / hn;
                ORC_PAR_FOR
                for (int t = 0; t < n; t++) vn[t] = hinv * w[t];
            } else {
                for (int t = 0; t < n; t++) vn[t] = 0.0;
            }
            for (k = 0; k < i; k++)
                orc_apply_rot(&H[k + i * (m + 1)], &H[(k + 1) + i * (m + 1)], cs[k], sn[k]);
            orc_gen_rot(H[i + i * (m + 1)], H[(i + 1) + i * (m + 1)], &cs[i], &sn[i]);
            orc_apply_rot(&H[i + i * (m + 1)], &H[(i + 1) + i * (m + 1)], cs[i], sn[i]);
            orc_apply_rot(&s[i], &s[i + 1], cs[i], sn[i]);
            done_iters++;
            resid = fabs(s[i + 1]) / normb;
            hist_push(&hs, resid);
            if (resid < *tol) {                                        /* "<" :654 */
                update(acc, i, H, m, s, V, n);
                if (op->kind == 1) orc_split_right(op->sp, y, x);     /* :2176 */
                *tol = resid;
                *max_iter = j;
                ret = 0;
                goto out;
            }
        }
        /* Update(m-1) in the reference even when j>max_iter cut the cycle
         * short (src/gmres.cu:677,2196); the restatement uses the last filled
         * column i-1 (deliberate fix, as ILU++ does). */
        update(acc, i - 1, H, m, s, V, n);
        if (op->kind == 1) orc_split_right(op->sp, y, x);
        orc_residual(n, op->rp, op->ci, op->v, x, b, rr);
        if (op->kind == 0)
            orc_lusolve(n, op->l_rp, op->l_ci, op->l_v, op->u_rp, op->u_ci, op->u_v, rr, r);
        else
            orc_split_left(op->sp, rr, r);
        beta = norm2(r, n);
        resid = beta / normb;
        hist_push(&hs, resid);
        if (resid < *tol) {
            *tol = resid;
            *max_iter = j;
            ret = 0;
            goto out;
        }
    }
    *tol = resid;
    ret = 1;
out:
    if (hist_len) *hist_len = hs.len < hist_cap ? hs.len : hist_cap;
    if (inner_iters) *inner_iters = done_iters;
    free(s); free(cs); free(sn); free(w); free(ww); free(r); free(rr); free(bb);
    free(H); free(V); free(y); free(s_cgs);
    return ret;
}

int orc_gmres_left(int n, const int *rp, const int *ci, const double *v,
                   const int *l_rp, const int *l_ci, const double *l_v,
                   const int *u_rp, const int *u_ci, const double *u_v,
                   const double *b, double *x, int m, int *max_iter, double *tol,
                   double *hist, int hist_cap, int *hist_len, int *inner_iters)
{
    op_t op = {0, n, rp, ci, v, l_rp, l_ci, l_v, u_rp, u_ci, u_v, NULL};
    return gmres_core(&op, b, x, m, max_iter, tol, hist, hist_cap, hist_len, inner_iters);
}

int orc_gmres_split(int n, const int *rp, const int *ci, const double *v,
                    const orc_split_t *p,
                    const double *b, double *x, int m, int *max_iter, double *tol,
                    double *hist, int hist_cap, int *hist_len, int *inner_iters)
{
    op_t op = {1, n, rp, ci, v, NULL, NULL, NULL, NULL, NULL, NULL, p};
    return gmres_core(&op, b, x, m, max_iter, tol, hist, hist_cap, hist_len, inner_iters);
}

/* ---------------------------------------------------------------- transient */
double orc_pulse(const double *q, int it, double h)
{
    const double vlo = q[0], vhi = q[1], td = q[2], tr = q[3], tf = q[4], tw = q[5], tp = q[6];
    double t = it * h;                         /* mytime = idxt * tstep */
    t = t - floor(t / tp) * tp;
    if (t < td) return vlo;
    if (t < td + tr) return vlo + (t - td) * (vhi - vlo) / tr;
    if (t < td + tr + tw) return vhi;
    if (t < td + tr + tw + tf) return vhi - (t - td - tr - tw) * (vhi - vlo) / tf;
    return vlo;
}

/* PWL source value at time index it (gen_PWLut_kernel, src/kernels.cu:146-176):
 * tv = {t0, v0, t1, v1, ...}, np points; value = v[i] - (t[i] - t)*(v[i] - v[i-1])
 * / (t[i] - t[i-1]) at the first i with t < t[i], v[np-1] after the last point.
 * Deviation: for t < t[0] the reference reads v[-1], t[-1] (out of bounds);
 * here the value is v[0] (the waveform holds its first point). */
double orc_pwl(const double *tv, int np, int it, double h)
{
    const double t = it * h;                   /* mytime = idxt * tstep */
    if (np <= 0) return 0.0;
    double value = tv[1];
    int i;
    for (i = 0; i < np; i++) {
        if (t < tv[2 * i]) {
            if (i > 0)
                value = tv[2 * i + 1] - (tv[2 * i] - t) * (tv[2 * i + 1] - tv[2 * i - 1]) /
                                            (tv[2 * i] - tv[2 * i - 2]);
            break;
        }
    }
    if (i == np) value = tv[2 * np - 1];
    return value;
}

void orc_transient_rhs(int n, int nsrc, const int *src_node, const double *u,
                       const double *cdiag, const double *x, double *w)
{
    for (int i = 0; i < n; i++) w[i] = 0.0;
    for (int k = 0; k < nsrc; k++) w[src_node[k]] += 1.0 * u[k];   /* cs_dl_gaxpy(B, u, w) */
    for (int i = 0; i < n; i++) {
        double xnr = 0.0;
        xnr += cdiag[i] * x[i];                                     /* cs_dl_gaxpy(right, xn, xnr) */
        w[i] += xnr;                                                /* w += xnr */
    }
}

/* cs_dl_gaxpy (CXSparse, called by the step driver at
 * src/mna_solve_gpu_gmres.cpp:585-591): y += A x for A in compressed columns,
 * column by column -- each y[i] accumulates its terms in column order */
void orc_gaxpy_csc(int ncol, const long *p, const long *i, const double *ax, const double *x, double *y)
{
    for (int j = 0; j < ncol; j++)
        for (long k = p[j]; k < p[j + 1]; k++) y[i[k]] += ax[k] * x[j];
}

/* ------------------------------------------------ sharded solve (oracle/dd.py)
 * One row of a triangular solve in the reference's arithmetic
 * (LUSolve_ignoreZero, src/SpMV_compute.cpp:92-136): x[r] = b[r], then
 * x[r] -= v_k * x[c_k] for the listed terms in order, then x[r] /= d[r]
 * (d = 1 for the unit / skipped diagonal: exact).  Rows ascending (lower) or
 * descending (upper).  sub_seq: the same subtraction without the division,
 * for the coupling terms a row subtracts before its own triangle's. */
void orc_canon_trsv(int n, int lower, const int *rp, const int *ci, const double *v,
                    const double *d, const double *b, double *x)
{
    for (int t = 0; t < n; t++) {
        const int r = lower ? t : n - 1 - t;
        double acc = b[r];
        for (int k = rp[r]; k < rp[r + 1]; k++) acc -= v[k] * x[ci[k]];
        x[r] = acc / d[r];
    }
}

void orc_sub_seq(int n, const int *rp, const int *ci, const double *v, const double *x,
                 const double *in, double *out)
{
    for (int r = 0; r < n; r++) {
        double acc = in[r];
        for (int k = rp[r]; k < rp[r + 1]; k++) acc -= v[k] * x[ci[k]];
        out[r] = acc;
    }
}
