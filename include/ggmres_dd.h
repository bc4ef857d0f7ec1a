/*
 * ggmres_dd.h -- C ABI of the sharded (domain-decomposed) GMRES solve, SURVEY.md 8(e).
 *
 * Replaces the reference's multi-domain path: partition4 (src/partition3.cpp:122-194,
 * METIS_PartGraphRecursive -> our recursive BFS bisection / contiguous blocks),
 * dd_form's arrow-matrix blocks (src/form_dd.cpp:32-110) and the per-domain
 * solves of etbr_dd (src/etbr_dd.cpp), here as ONE GMRES(m) + ILU(0) solve of
 * the arrow-permuted system B = P A P^T sharded over nparts GPUs:
 *
 *   - shard p holds interior p's rows and a replica of the separator rows;
 *   - SpMV and the forward triangular solve need the "interface" values
 *     (interior nodes the separator rows reference) of every shard: one
 *     all-gather each (RCCL over xGMI); the backward solve needs nothing;
 *   - every MGS dot is an all-gather of the shards' block partials, summed in
 *     one fixed order on every shard (identical Hessenberg on every shard);
 *   - the ILU(0) factors are those of B (factored on the host), and each row
 *     of every triangular solve runs the reference's operations in the
 *     reference's order (LUSolve_ignoreZero, src/SpMV_compute.cpp:92-136):
 *     the operators are bit-identical to the single-GPU solve of B.
 *
 * Three communicators:
 *   GG_DD_RCCL   one process per GPU (torchrun), shard = rank, RCCL collectives
 *                on the solver's stream; the 128-byte id comes from
 *                gg_dd_unique_id on rank 0 and is broadcast by the caller.
 *   GG_DD_IPC    one process per shard, device-initiated exchanges: every
 *                rank's exchange area (uncached device memory) is mapped into
 *                every process (hipIpc; over xGMI between GPUs) and each
 *                all-gather is ONE small kernel that stores this rank's slot
 *                into every peer's area and waits on the peers' sequence-
 *                numbered flags -- no collective library.  Several ranks may
 *                share a GPU (the one-GPU test of the multi-process path).
 *                Bootstrap: gg_dd_create, gg_dd_ipc_handle, the caller
 *                all-gathers the nparts handles (any host channel), then
 *                gg_dd_ipc_connect before gg_dd_set_system.
 *   GG_DD_LOCAL  all nparts shards in this process on one device (the same
 *                kernels, the exchanges done by a copy kernel): tests and
 *                single-GPU studies of the decomposition.
 *
 * Vectors are global, natural (unpermuted) order, length n, identical on every
 * rank on input.  On output a process writes the rows it holds (GG_DD_LOCAL:
 * all rows; GG_DD_RCCL / GG_DD_IPC: interior p and the separator); other
 * entries are left untouched.  Status codes as ggmres.h; GG_ECOMM for RCCL
 * failures, GG_ETIMEOUT when an IPC peer does not arrive within 30 s.
 */
#ifndef GGMRES_DD_H_
#define GGMRES_DD_H_

#include "ggmres.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GG_DD_ID_BYTES 128

#define GG_DD_IPC_HANDLE_BYTES 64

enum gg_dd_comm {
    GG_DD_LOCAL = 0,
    GG_DD_RCCL = 1,
    GG_DD_IPC = 2,
    /* timing only: ONE process holds shard `rank` of nparts and every exchange
     * is the in-process all-gather kernel over its own buffer (the other
     * shards' slots keep stale values) -- the per-rank kernel and exchange-launch
     * time of a one-shard-per-GPU run on this device alone.  The solve's values
     * are NOT the system's: run it for a fixed iteration count. */
    GG_DD_LOOPBACK = 3
};

typedef struct gg_dd gg_dd;

/* ncclGetUniqueId: call on rank 0, broadcast the bytes to every rank */
int gg_dd_unique_id(unsigned char *id);
int gg_dd_create(int device, int nparts, int comm, int rank, const unsigned char *id, gg_dd **out);
int gg_dd_destroy(gg_dd *d);
/* GG_DD_IPC: this rank's exchange-area handle (GG_DD_IPC_HANDLE_BYTES) ... */
int gg_dd_ipc_handle(gg_dd *d, unsigned char *handle);
/* ... and every rank's, rank-major (nparts * GG_DD_IPC_HANDLE_BYTES): maps the
 * peers' areas; returns once every rank has connected */
int gg_dd_ipc_connect(gg_dd *d, const unsigned char *handles);
/* processes in the exchange: GG_DD_RCCL the communicator's rank count
 * (ncclCommCount), GG_DD_IPC the mapped areas (checked: every rank reports
 * its own rank), GG_DD_LOCAL 1; *rank = this process's rank */
int gg_dd_comm_ranks(gg_dd *d, int *ranks, int *rank);

/* the global system (identical on every rank): partition (gg_part_method of
 * ggmres_host.h), arrow permutation, ILU(0) of the permuted matrix, shards */
int gg_dd_set_system(gg_dd *d, int n, const int *row_ptr, const int *col_idx, const double *val,
                     int method);
/* info[0..9] (exactly 10 ints): n, nparts, separator rows, max interface per
 * shard, this process's first shard: interior rows, interior solves (0
 * level-scheduled, 2 / 3 the 2D / 3D wavefront), separator solves (0
 * level-scheduled launches, 1 the fused separator step, 2 / 3 wavefront),
 * local vector length (slots), shards in this process, halo doubles exchanged
 * per all-gather (received, per shard) */
int gg_dd_info(gg_dd *d, int *info);
/* *on = 1 when the orthogonalization runs with its exchanges inside its
 * kernels (GG_DD_IPC / GG_DD_LOOPBACK, P > 1, environment GG_DD_XK=1 at
 * gg_dd_create; measured slower than the default), else 0 */
int gg_dd_xk_active(gg_dd *d, int *on);
/* the arrow permutation in use: pinv[j] = new index of node j; q = its inverse */
int gg_dd_perm(gg_dd *d, int *pinv, int *q);

/* the reduction order of the shard's dots (for order-matched parity checks):
 * out[slot] = permuted row of each slot of the part's dot range (-1 = padding),
 * G = block partials per shard; returns the range length (part must be held
 * by this process) */
int gg_dd_dot_layout(gg_dd *d, int part, long long *out, long long cap, int *G);

int gg_dd_solve(gg_dd *d, const double *b, double *x, const gg_options *opt, gg_result *res);
int gg_dd_solve_device(gg_dd *d, const double *d_b, double *d_x, const gg_options *opt,
                       gg_result *res);
int gg_dd_get_history(gg_dd *d, double *out, int cap);

/* single operators (host vectors, natural order) for parity tests */
int gg_dd_spmv(gg_dd *d, const double *x, double *y);
int gg_dd_precond_apply(gg_dd *d, const double *in, double *out);
/* division in the shards' wavefront triangular solves (ggmres.h gg_set_division:
 * GG_DIV_FMA fuses the rows of the interiors' unskewed 2D-grid wavefronts, the
 * other wavefronts multiply as GG_DIV_RCP; the separator's solves divide) */
int gg_dd_set_division(gg_dd *d, int mode);
/* average device time (hipEvents on the solver's stream, microseconds) of one
 * all-gather of cnt doubles per shard over this communicator -- the exchange
 * every sharded operator and dot pays (cnt <= (m+1) * G of the last solve) */
int gg_dd_time_exchange(gg_dd *d, long long cnt, int reps, double *avg_us);
/* In-solve timing of the sharded solve's families per inner iteration
 * (hipEvent pairs on the solver's stream, accounted for the iterations that
 * really ran): the interior rows' + separator rows' SpMV with its halo
 * exchange, the interior L solve, the separator step (interface exchange and
 * separator solves), the interior U solve, the orthogonalization (its
 * exchanges included).  kinds: a mask of (1 << GG_DD_PROF_*). */
enum gg_dd_prof_kind {
    GG_DD_PROF_SPMV = 0, GG_DD_PROF_TRSV_L = 1, GG_DD_PROF_SEP = 2, GG_DD_PROF_TRSV_U = 3,
    GG_DD_PROF_ORTH = 4, GG_DD_PROF_NKINDS = 5
};
int gg_dd_profile_enable(gg_dd *d, int kinds);
int gg_dd_profile_reset(gg_dd *d);
int gg_dd_profile_get(gg_dd *d, int kind, int *launches, double *total_ms);
/* algorithmic bytes of one launch of family `kind`
 * (GG_DD_PROF_SPMV / _TRSV_L / _TRSV_U) over the shards of this process */
int gg_dd_bytes(gg_dd *d, int kind, double *bytes);

#ifdef __cplusplus
}
#endif
#endif
