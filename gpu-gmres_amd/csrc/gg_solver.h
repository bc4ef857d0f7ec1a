// gg_solver.h -- the single-device solver object behind the C ABI (solver.hip)
// and the many-RHS batch driver (batch.hip).
#pragma once

#include <vector>

#include "kernels.h"

namespace gg {
struct BatchWs;                       // batch.hip
void batch_release(gg_solver *s);     // frees s->batch (gg_destroy)
// solver.hip: one single-scenario device solve (gg_solve_device's engine, with
// its fallbacks) and the padding map of the solver's vector space
int solve_one(gg_solver *s, const double *d_b, double *d_x, const gg_options *opt, gg_result *res);
UnitMap solver_unit_map(const gg_solver *s);
// batch.hip: the many-RHS engine behind gg_solve_batch_device
int solve_batch(gg_solver *s, int S, const double *d_b, long long ldb, double *d_x, long long ldx,
                const gg_options *opt, gg_result *res);
bool batch_engine_on(gg_solver *s);
long long batch_history(gg_solver *s, int q, double *out, long long cap);
}  // namespace gg

using gg::Csr;
using gg::DBuf;
using gg::DevCsr;
using gg::DevState;
using gg::DevTri;
using gg::Wave2D;

struct gg_solver {
    int device = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;

    Csr A;
    bool have_A = false;
    int pkind = -1;       // -1: not set

    // vector space (natural or wavefront layout)
    bool wave = false;
    bool relabeled = false;   // off the wavefront, an RCM layout (setup_space)
    Wave2D wl;
    long long P = 0, Ppad = 0;
    std::vector<long long> nat2lay_h;
    DBuf<long long> lay2nat, nat2lay;
    int G = 1;

    DevCsr dA;            // A in layout space (split: A' -- rows in prow order, columns by pcol)
    DevTri L, U;
    // Split (PG) engine, every vector in the triangles' layout (natural or
    // wavefront).  With lay = the layout map of the triangles' row space:
    //   A'  row lay(j) = A row prow[j], column c -> lay(pcol[c])
    //   mid_l[lay(r)] = middle[r], ls_l[lay(j)] = lscale[prow[j]],
    //   rs_l[lay(r)] = rscale[pcol^-1[r]]   (all three 1.0 in padding slots)
    // so that Ml(A Mr(v)) = L^-1 (A' (U^-1 (mid_l o v) / rs_l)) / ls_l with the
    // row gather, the column scatter and both scalings folded into the SpMV's
    // indices and epilogue and the U solve's store (each value rounded by the
    // same operation as in MyILUPPfloat::DevPrecond_*, src/preconditioner.cu:
    // 1424-1657).  x lives in the same column convention: x[c] at lay(pcol[c]).
    DBuf<double> mid_l, ls_l, rs_l;
    // stage maps (layout slot -> natural index, -1 = padding): b in A' row
    // order, x in the column convention; and back: x_out[c] = lay(pcol[c]),
    // y_out[r] = lay(prow^-1[r])
    DBuf<long long> sb_map, sx_map, sx_out, sy_out;
    DevCsr dUfull;        // the split U factor (diagonal first) in layout space (apply_start)
    // caller-supplied preconditioner (gg_set_precond_user): fp32 staging of its
    // device arrays, natural order
    gg_precond_fn ufn = nullptr;
    void *uctx = nullptr;
    DBuf<float> fin, fout;

    // workspace
    int m_alloc = -1;
    DBuf<double> V, w, ww, r, rr, bb, t1, t2, z, xv, bv, y;
    DBuf<double> partA, partB, H, s, cs, sn, ysm;
    // persistent Arnoldi orthogonalization (kernels.hip k_arnoldi_persist)
    bool persist = false;
    bool split_local = false;   // the split engine's vectors in a local layout (grid / RCM): its gathers are near
    bool wide = false;                  // k_arnoldi_wide (vectors beyond persist's registers)
    bool shared = false;                // GG_SOLVE_SHARED_DEVICE for the solve in progress
    int div_mode = GG_DIV_EXACT;        // gg_set_division: the wavefront solves' division
    // pinned host copies of the control block and the error word (one
    // round trip per restart cycle reads both)
    DevState *h_state = nullptr;
    int *h_err = nullptr;
    // the pipelined cycle loop: two pinned slots, each the state after one cycle
    DevState *p_state[2] = {nullptr, nullptr};
    int *p_err[2] = {nullptr, nullptr};
    hipEvent_t p_ev[2] = {nullptr, nullptr};
    std::vector<size_t> mark_ends;      // marks.size() after each enqueued cycle (pipelined)
    int resid_fallbacks = 0;            // cycles rerun after a persistent grid was not co-resident
    int iter_hint = 0;                  // transient loop: the previous step's inner iterations (0: none)
    // transient tap-node statistics (gg_transient_set_taps / _get_taps)
    std::vector<int> taps;
    std::vector<double> tap_max, tap_min, tap_avg;
    DBuf<unsigned long long> gran;      // m * (m+2) * G hand-off granules, then m * (m+2) sums
                                        // (gather_h), re-armed per cycle
    DBuf<unsigned long long> xgran;     // m * (m+2) * kMgsXcdWords: the XCD-local gather's slots (re-armed per cycle)
    DBuf<unsigned long long> elect;     // per XCD: the last launch that elected its reducer
    unsigned long long mgs_seq = 0;     // persistent orthogonalization launches so far (election)
    DBuf<long long> mgs_trace;          // diagnostics: GG_MGS_TRACE=N stamps the N-th persistent launch
    int mgs_trace_i = -1;               // (its inner index; printed to stderr after the solve)
    DBuf<double> hist;
    long long hist_cap = 0;
    DBuf<DevState> ds;
    DBuf<int> err;
    DBuf<double> nat_in, nat_out;   // staging for host-vector entry points
    std::vector<double> last_hist;

    // in-solve kernel timing (gg_profile_*)
    int prof_mask = 0;                  // (1 << GG_PROF_*) bits being timed
    std::vector<hipEvent_t> prof_pool;
    size_t prof_used = 0;
    std::vector<int> prof_free;         // pool slots of collected marks, reusable
    struct Mark { int kind, i, e0, e1; };
    std::vector<Mark> marks;
    double prof_ms[GG_PROF_NKINDS] = {};
    long long prof_cnt[GG_PROF_NKINDS] = {};

    // the many-RHS solve's per-scenario arenas (batch.hip), kept between
    // batched solves of the same shape
    gg::BatchWs *batch = nullptr;
};
