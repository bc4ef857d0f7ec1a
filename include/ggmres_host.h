/*
 * ggmres_host.h -- host-only (no GPU) setup entry points of libggmres.so.
 *
 * The setup phase of the reference path runs on the host; these entry points
 * expose the product's implementation of it so it can be checked (and used)
 * without a device:
 *   gg_host_ilu0   leftILU            src/leftILU.cu:27-336
 *   gg_host_iluk   ilukC + lofC       src/iluk.cpp:56-334
 *   gg_host_wave2d / gg_host_wave3d
 *                  structured-grid detection for the wavefront SpTRSV
 *                  (replaces cusparseScsrsv_analysis, src/gmres.cu:1516-1517)
 *   gg_host_partition  partition4      src/partition3.cpp:122-194 (METIS is not
 *                  available: recursive BFS bisection or contiguous blocks)
 *   gg_host_permute    the arrow permutation P A P^T of the DD solve
 *   gg_host_block      dd_form block extraction  src/form_dd.cpp:32-110
 *   gg_host_read_mtx   readSparseMatrix (Matrix Market)  src_thermal/SpMV_gen.cpp:93-187
 *   gg_host_coo2csr_in coo2csrDouble_in  src/formatConvert.cpp:165-216
 *   gg_host_read_netlist  SPICE power-grid netlist -> MNA (G, C, B, sources):
 *                  parser() + stampG/stampC/stampB  src/parser.cpp:69-272, 1904-2886
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
/* The ILU(level) pattern as flat rows (each row ascending, diagonal included):
 * lofC's level-of-fill pattern (src/iluk.cpp:193-334), built row-parallel over
 * `threads` host threads -- level 1 by the original L x U entries, level >= 2
 * by incomplete fill paths; prow[n+1] caller-allocated, *pcol
 * malloc'd (gg_host_free).  The symbolic phase of gg_set_precond_iluk_device. */
int gg_host_iluk_pattern(int level, int n, const int *row_ptr, const int *col_idx, int threads,
                         int *prow, int **pcol);
/* For ILU factors (L unit-lower diag last, U diag first): 1 and the grid
 * line length / count if the wavefront path applies, else 0. */
int gg_host_wave2d(int n, const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                   const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                   int *nx, int *ny);
enum gg_part_method {
    GG_PART_BISECT = 0,    /* recursive BFS bisection of the node graph (METIS stand-in) */
    GG_PART_BLOCKS = 1,    /* contiguous index ranges (strips / slabs of a natural-order grid) */
    GG_PART_GRID = 2,      /* px x py rectangles of a natural-order 2D grid (px the largest divisor
                              of nparts <= sqrt(nparts); line length = the pattern's most frequent
                              |offset| > 1): rectangular interiors, shorter wavefront chains */
    GG_PART_COLOR_SEP = 4  /* flag (extension): separator ordered by a greedy colouring of its
                              graph, then by index, instead of by index alone */
};
/* nparts interiors + the separator part `nparts` (every endpoint of a cut edge
 * of the symmetrized pattern).  node_part[n]; part_size[nparts + 1];
 * pinv[j] = new index of node j; q[i] = node at new index i (interiors first,
 * separator last, ascending original index inside a part). */
int gg_host_partition(int n, const int *row_ptr, const int *col_idx, int nparts, int method,
                      int *node_part, int *part_size, int *pinv, int *q);
/* B = P A P^T for (pinv, q) of gg_host_partition; a row's entries sorted by
 * new column (stable) */
int gg_host_permute(int n, const int *row_ptr, const int *col_idx, const double *val,
                    const int *pinv, const int *q,
                    int *b_row_ptr, int **b_col_idx, double **b_val);
/* rows [r0, r1) x columns [c0, c1) of a CSR (As_k, E_k, F_k, At of dd_form
 * are the blocks of B at the part boundaries); b_row_ptr has r1 - r0 + 1 slots */
int gg_host_block(int n, const int *row_ptr, const int *col_idx, const double *val,
                  int r0, int r1, int c0, int c1,
                  int *b_row_ptr, int **b_col_idx, double **b_val);
/* Matrix Market coordinate file -> CSR (0-based, entries sorted by (row, col),
 * stable: duplicates kept in file order, as readSparseMatrix keeps them).
 * The reference reads every file as general; expand_symmetric != 0 mirrors
 * the strict triangle of symmetric / skew-symmetric files (an extension).
 * 'pattern' files get value 1.  Values are parsed as fp64 (the reference
 * narrows to float).  Returns GG_OK or GG_EINVAL (unreadable / malformed). */
int gg_host_read_mtx(const char *path, int expand_symmetric, int *nrows, int *ncols,
                     int **row_ptr, int **col_idx, double **val);
/* the same for a 3D 7-point grid (offsets nx*ny, nx, 1): 1 and the grid
 * dimensions if the 3D wavefront path applies, else 0 */
int gg_host_wave3d(int n, const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                   const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                   int *nx, int *ny, int *nz);
/* The wavefront vector layout the solver would use for these factors (no
 * device needed): returns 1 and fills slot[r] (natural row -> layout slot,
 * n entries, may be NULL) and info[9] = {kind (2: 2D bands, 3: 3D tiles,
 * 4: 3D planes), nx, ny, nz, bands or tiles, steps per band T, tiles along
 * the lines NJ / planes NK, lane skew}; 0 when the layout is natural.
 * Replaces the level analysis cusparseScsrsv_analysis (src/gmres.cu:1516-1517)
 * for grid-shaped triangles (kernels.hip k_trsv_wave2d / k_trsv_tile3d). */
int gg_host_wave_layout(int n, const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                        const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                        long long *slot, int *info);
/* The same for the split (ILU++) factors of gg_set_precond_split (L diagonal
 * last, U diagonal first; the PG path's MyILUPP::HostPrecond_left/_right,
 * src/preconditioner.cu:1094-1137): info[0] = 2 (2D bands) or 5 (bordered
 * grid: the first info[6] rows -- an MNA system's pads and voltage-source
 * branches -- at slots [0, info[6]), the grid rows at info[7] + their 2D
 * slot), info[1..5] = nx, ny, nz, bands, T) or 6 (off the wavefront: the flow
 * kernel's RCM layout, slot[r] = r's position in a reverse Cuthill-McKee order
 * of the factors' pattern).  0 when the layout is natural (GG_FLOW_RCM=0).
 * The solver's environment overrides apply here too (GG_NO_WAVEFRONT=1: no
 * wavefront; GG_NO_BORDER=1: no bordered grid). */
int gg_host_split_layout(int n, const int *l_row_ptr, const int *l_col_idx, const double *l_val,
                         const int *u_row_ptr, const int *u_col_idx, const double *u_val,
                         long long *slot, int *info);
/* coo2csrDouble_in (src/formatConvert.cpp:165-216): COO -> CSR in place;
 * on return row_idx[0..nrows] holds the row pointers (row_idx needs
 * max(nz, nrows + 1) slots), entries of a row bubble-sorted by column.
 * The reference's C++ boundary-feed symbols are in include/compat/format_convert.h. */
int gg_host_coo2csr_in(int nrows, int nz, double *val, int *row_idx, int *col_idx);
/* Flat SPICE power-grid netlist (R, C, L, V, I element lines, '+' PWL
 * continuation lines, .tran tstep tstop, .print/.probe ports, one .include
 * level) -> the reference's MNA system.  Unknowns: the n_nodes non-ground
 * nodes numbered by first appearance ("0" and "gnd" are ground), then one
 * branch current per inductor and per voltage source, n in all.
 *   G (n x n): R stamps 1/R; L and V branch incidences +-1
 *   C (n x n): C stamps; L branch rows get L
 *   B (n x (n_v + n_i)): V source k: -1 at its branch row; I source k:
 *                        -1 at n1, +1 at n2
 * CSR, columns ascending, duplicate stamps summed in netlist order (as the
 * reference's matrix::pushEntry).  Source k (V first, then I, netlist order):
 * src_kind[k] in gg_src_kind, parameters src_data[src_ptr[k] .. src_ptr[k+1]):
 * DC {value}; PULSE {v1, v2, td, tr, tf, pw, period} from "<dc> PULSE(...)"
 * (gen_PULSEut_kernel's parameters); PWL {t0, v0, t1, v1, ...} with a point
 * (0, v0) in front when t0 != 0.  port[k] = unknown index of .print port k
 * (-1: ground or unknown name).  Arrays are malloc'd; release the whole
 * struct with gg_host_free_netlist.  GG_EINVAL if the file cannot be read.
 * Deliberate deviation: an R/C/L/V/I line without a name, two nodes and a
 * value rejects the netlist (GG_EINVAL, gg_last_error names the line); the
 * reference prints "Fail in obtaining ... value" and skips the stamp but still
 * counts the V / L branch row (src/parser.cpp:746-762, 854-858), leaving an
 * all-zero row in G (tests/test_netlist.py::test_netlist_short_element_line_rejected). */
typedef struct gg_netlist {
    int n_nodes, n_l, n_v, n_i, n;
    double tstep, tstop;
    int *g_row_ptr, *g_col_idx;
    double *g_val;
    int *c_row_ptr, *c_col_idx;
    double *c_val;
    int *b_row_ptr, *b_col_idx;
    double *b_val;
    int *src_kind, *src_ptr;
    double *src_data;
    int nport;
    int *port;
} gg_netlist;
int gg_host_read_netlist(const char *path, gg_netlist *out);
void gg_host_free_netlist(gg_netlist *nl);
/* Sharded-solve plan (the host half of include/ggmres_dd.h, exposed for CPU
 * checks of the decomposition): partition4 + arrow permutation B = P A P^T +
 * ILU(0) of B + per-part pieces in the part's local index space
 * [interior (nI) | separator (nS) | halo (nparts * max_iface)]. */
typedef struct gg_dd_plan gg_dd_plan;
enum gg_dd_piece {
    GG_DD_A = 0,      /* local rows of B, local columns                          */
    GG_DD_LI = 1,     /* interior triangle L_II (canonical order, off-diagonals)  */
    GG_DD_LS = 2,     /* separator triangle L_SS                                  */
    GG_DD_LSH = 3,    /* separator rows' interior terms of L (cols: halo index)   */
    GG_DD_UI = 4,     /* interior triangle U_II                                   */
    GG_DD_US = 5,     /* separator triangle U_SS                                  */
    GG_DD_UIS = 6     /* interior rows' separator terms of U (cols: separator idx)*/
};
int gg_host_dd_plan(int n, const int *row_ptr, const int *col_idx, const double *val, int nparts,
                    int method, gg_dd_plan **out);
/* sizes[4]: n, nparts, separator rows, max interface nodes per part */
int gg_host_dd_plan_sizes(const gg_dd_plan *pl, int *sizes);
/* part_size[nparts + 1], pinv[n], q[n] (any may be NULL) */
int gg_host_dd_plan_perm(const gg_dd_plan *pl, int *part_size, int *pinv, int *q);
/* sizes[3]: nI, nS, number of own interface nodes */
int gg_host_dd_shard_sizes(gg_dd_plan *pl, int part, int *sizes);
/* a piece as CSR (row_ptr malloc'd too); triangles list the off-diagonal
 * terms in the reference's summation order */
int gg_host_dd_shard_csr(gg_dd_plan *pl, int part, int piece, int *nrows, int **row_ptr,
                         int **col_idx, double **val);
/* divisors of a triangle piece (GG_DD_LI/LS/UI/US), nrows doubles */
int gg_host_dd_shard_div(gg_dd_plan *pl, int part, int piece, double *d);
/* own interface nodes (interior-local, ascending) and the permuted global index
 * of every local row (nI + nS) (either may be NULL) */
int gg_host_dd_shard_index(gg_dd_plan *pl, int part, int *iface, int *rows);
void gg_host_dd_plan_free(gg_dd_plan *pl);
void gg_host_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
