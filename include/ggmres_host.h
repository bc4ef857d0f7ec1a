/*
 * ggmres_host.h -- host-only (no GPU) setup entry points of libggmres.so.
 *
 * The setup phase of the reference path runs on the host; these entry points
 * expose the product's implementation of it so it can be checked (and used)
 * without a device:
 *   gg_host_ilu0   leftILU            src/leftILU.cu:27-336
 *   gg_host_iluk   ilukC + lofC       src/iluk.cpp:56-334
 *   gg_host_wave2d structured-grid detection for the wavefront SpTRSV
 *                  (replaces cusparseScsrsv_analysis, src/gmres.cu:1516-1517)
 * Output arrays are malloc'd by the library; release them with gg_host_free.
 */
#ifndef GGMRES_HOST_H_
#define GGMRES_HOST_H_

#ifdef __cplusplus
extern "C" {
#endif

int gg_host_ilu0(int n, const int *row_ptr, const int *col_idx, const double *val,
                 int *l_row_ptr, int **l_col_idx, double **l_val,
                 int *u_row_ptr, int **u_col_idx, double **u_val);
int gg_host_iluk(int level, int n, const int *row_ptr, const int *col_idx, const double *val,
                 int *l_row_ptr, int **l_col_idx, double **l_val,
                 int *u_row_ptr, int **u_col_idx, double **u_val);
/* For ILU factors (L unit-lower diag last, U diag first): 1 and the grid
 * line length / count if the wavefront path applies, else 0. */
int gg_host_wave2d(int n, const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                   const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                   int *nx, int *ny);
void gg_host_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
