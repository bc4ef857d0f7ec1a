// gg_internal.h -- internal types of the MI355X GMRES solver (host + device).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ggmres.h"
#include "ggmres_host.h"

namespace gg {

// ------------------------------------------------------------------ errors
void set_error(const std::string &msg);
struct Error {
    int code;
    std::string msg;
};
#define GG_HIP(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            throw ::gg::Error{GG_EHIP, std::string(#call) + ": " + hipGetErrorString(e_) + \
                                           " @" + __FILE__ + ":" + std::to_string(__LINE__)}; \
    } while (0)
#define GG_REQUIRE(cond, code, msg)                                                    \
    do {                                                                               \
        if (!(cond)) throw ::gg::Error{code, msg};                                     \
    } while (0)

// ---------------------------------------------------------------- host CSR
struct Csr {
    int n = 0;
    std::vector<int> rp, ci;
    std::vector<double> v;
    int nnz() const { return rp.empty() ? 0 : rp[n]; }
};

// A triangular solve in "canonical" form: for each row r (in its solve order)
//   x[r] = (b[r] - sum_k off_v[k] * x[off_c[k]]) / d[r]
// with the off-diagonal terms listed in exactly the reference's summation
// order.  A unit or skipped diagonal is d = 1 (division by 1 is exact).
struct CanonTri {
    bool lower = true;
    Csr off;                 // off-diagonal entries, reference order
    std::vector<double> d;   // divisors
};

// host-side factorization (host/factor.cpp)
void ilu0_left(const Csr &A, Csr &L, Csr &U);                 // leftILU semantics
// domain decomposition setup (host/partition.cpp): partition4 with a recursive
// BFS bisection (or contiguous blocks) in place of METIS, the arrow permutation,
// dd_form's block extraction
void partition_arrow(const Csr &A, int nparts, int method, std::vector<int> &node_part,
                     std::vector<int> &part_size, std::vector<int> &pinv, std::vector<int> &q);
Csr arrow_permute(const Csr &A, const std::vector<int> &pinv, const std::vector<int> &q);
// GG_PART_GRID's shape: line length nx (the pattern's most frequent |offset| > 1),
// for a 3D grid the plane nx*ny (the most frequent multiple of nx above it, if
// >= n/8 entries), and px x py (x pz) = nparts blocks -- 2D: px the largest
// divisor <= sqrt; 3D: px <= py <= pz, the most cube-like; nx = 0 if A is not a
// natural-order grid of whole lines (planes) with room for the blocks
struct GridBlocks {
    int nx = 0, ny = 0, nz = 1, px = 0, py = 0, pz = 1;
};
void grid_blocks(const Csr &A, int nparts, GridBlocks &gb);
Csr csr_block(const Csr &A, int r0, int r1, int c0, int c1);
// Matrix Market reader (host/mtx.cpp; readSparseMatrix semantics, fp64)
bool read_mtx(const char *path, bool expand_symmetric, int &nrows, int &ncols, Csr &A);
// splitLU_csr (src/leftILU.cu:481-541): drop |v| < 1e-9, unit diagonal LAST in L
void split_lu_drop(const Csr &F, Csr &L, Csr &U);
// CSC pattern of a square CSR (rows ascending per column) and the position maps
// csc2csr[k] = CSR position of CSC entry k, csr2csc its inverse
void csc_pattern(const Csr &A, std::vector<int> &cp, std::vector<int> &ri,
                 std::vector<long long> &csc2csr, std::vector<long long> &csr2csc);
int iluk_itsol(const Csr &A, int lof, Csr &L, Csr &U);        // lofC + ilukC, 0 or GG_EZEROPIVOT
// its pieces: lofC's patterns (L part in leftmost-pivot order, U part in
// insertion order) and the emission of ilukC's factors in the solver's forms
void iluk_symbolic(const Csr &A, int lof, std::vector<std::vector<int>> &Lja,
                   std::vector<std::vector<int>> &Uja);
// ILU(k) pattern as flat ascending rows (L part, diagonal, U part); k = 1
// row-parallel over host threads (factor.cpp)
void iluk_pattern(const Csr &A, int lof, int threads, std::vector<long long> &prow, std::vector<int> &nl,
                  std::vector<int> &pcol);
void iluk_emit_flat(int n, const std::vector<long long> &prow, const std::vector<int> &nl,
                    const std::vector<int> &pcol, const std::vector<double> &val, Csr &L, Csr &U);
void iluk_emit(const std::vector<std::vector<int>> &Lja, const std::vector<std::vector<int>> &Uja,
               const std::vector<std::vector<double>> &Lma, const std::vector<std::vector<double>> &Uma,
               const std::vector<double> &Draw, Csr &L, Csr &U);

// canonical forms (host/analysis.cpp)
CanonTri canon_lower_unit(const Csr &L);        // LUSolve_ignoreZero forward (diag never applied)
CanonTri canon_upper_ignorezero(const Csr &U);  // LUSolve_ignoreZero backward
CanonTri canon_lower_lastdiag(const Csr &L);    // MyILUPP HostPrecond_left (divide by last)
CanonTri canon_upper_firstdiag(const Csr &U);   // MyILUPP HostPrecond_right (divide by first)

// ---- sharded (domain-decomposed) solve: host plan (host/dd_setup.cpp) ----
constexpr int kMaxShards = 16;
struct DDPlan {
    int n = 0, P = 0;
    std::vector<int> part_size, pinv, q, begin;   // partition4 sizes / permutation, part offsets (P+2)
    Csr B;                                        // arrow-permuted A
    CanonTri cl, cu;                              // canonical ILU(0) triangles of B
    std::vector<std::vector<int>> iface;          // per part: interface nodes (permuted index)
    std::vector<int> hidx;                        // permuted index -> halo index, -1 if none
    int maxI = 0;
};
// one part's pieces in its local index space [interior | separator | halo]
struct DDShardHost {
    int p = 0, nI = 0, nS = 0;
    Csr A;                      // nI + nS rows, local columns
    CanonTri LI, LS, UI, US;    // region triangles (region-local indices)
    Csr LSH;                    // nS rows: interior terms of separator L rows (cols = halo index)
    Csr UIS;                    // nI rows: separator terms of interior U rows (cols = separator index)
    std::vector<int> iface;     // own interface nodes, interior-local, ascending
    std::vector<int> rows;      // permuted global index of each local row
};
DDPlan dd_plan(const Csr &A, int P, int method);
DDShardHost dd_shard(const DDPlan &D, int p);

// level sets for a canonical triangle: rows grouped by dependency depth
struct Levels {
    std::vector<int> ptr;    // nlev+1
    std::vector<int> rows;   // n
};
// ext_cols: columns >= n (an upper tail's references into the bordered grid,
// solved before it) are ignored rather than rejected
Levels level_sets(const CanonTri &T, bool ext_cols = false);
// Reverse Cuthill-McKee order of the symmetric pattern of the two triangles
// (order[k] = the row placed at slot k): the layout of the flow-kernel path
// (gg_set_precond_split off the wavefront), so that the rows of a level task
// and their terms' x sit close together in memory.  Deterministic: BFS from a
// pseudo-peripheral node of each component (lowest degree, then index),
// neighbours by (degree, index).
std::vector<int> rcm_order(const CanonTri &L, const CanonTri &U);
// T in the layout space of nat2lay (a permutation of the rows): row p = row
// nat(p) with its columns mapped, term order kept; levels from the natural
// triangle, each level's rows in ascending slot order
void relabel_tri(const CanonTri &C, const std::vector<long long> &nat2lay, CanonTri &out, Levels &lv);

// 2D structured-grid wavefront layout (SURVEY.md 7 hard parts)
//   natural row r = j*nx + i, band = j/64, lane l = j%64, step t = i + l:
//   slot = ((band*(T/2) + t/2)*64 + l)*2 + t%2     (a lane's step pair adjacent)
//   T = nx + 63 rounded up to a multiple of 64 (four 16-step kernel batches)
// steps per band are padded to a multiple of this (whole batches, an even
// number of them for the two-deep boundary polls; kernels.hip checks it)
constexpr int kWaveTAlign = 32;
// 3D tiles: steps per tile padded to whole pairs of 8-step batches (k_trsv_tile3d)
constexpr int kTileTAlign = 16;
constexpr int kTileDummyBlocks = 2048;   // workgroups with their own dummy granules (grid cap)
struct Wave2D {
    bool ok = false;
    int nx = 0, ny = 0, nz = 1, nbands = 0, T = 0;
    // lines lag each other by `skew` steps (1: ILU(0); k+1: ILU(k) on a 5-point
    // grid, whose rows also reference (j-1, i+a), a <= k); 2D only.  Row (j, i)
    // runs at step t = i + skew*l + (skew-1): the skew-1 lead-in steps fill the
    // edge lane's history of the neighbour band's line (forward), and T keeps
    // as many after the last row (backward)
    int skew = 1;
    // the upper triangle's rows list the in-line term (r+1) before the line term
    // (r+nx): the split (ILU++) U factor's ascending order (detect_wave2d's
    // split_u); 2D, skew 1 only
    bool u_inline_first = false;
    long long P2 = 0;        // one plane's layout length (nbands * T * 64)
    long long P = 0;         // padded layout length (nz * P2)
    // 3D tile layout (tile = true; kernels.hip k_trsv_tile3d): a wave owns a
    // tile of 8 lines x 8 planes, lane l = a + 8*g(c) for line j = 8J + a,
    // plane k = 8K + c, with the Gray code g(c) = c ^ (c >> 1): consecutive
    // planes sit in half-rows that differ in one bit, i.e. one DPP row_ror:8,
    // v_permlane16_swap or v_permlane32_swap apart.  Point (i, j, k) runs at
    // step t = i + a + c of its tile (a plane lags its predecessor by 1 step, as a
    // line lags its neighbour line: the DAG's own skew; round 2 used 2 steps,
    // so the cross-lane move is off the recurrence); tiles K-major (band =
    // K*NJ + J), each stored as a 2D band of T steps (nbands = NJ * NK; nz
    // stays the grid's plane count).
    bool tile = false;
    int NJ = 0, NK = 0;           // tiles along the line / plane directions
    // bordered grid (detect_border2d; 2D, skew 1): the first `bnt` rows are a
    // tail of non-grid rows (an MNA system's pad nodes and voltage-source
    // branch currents, pivoted ahead of the mesh) at slots [0, bnt); grid row
    // r >= bnt at bofs + its 2D slot.  P covers both.
    int bnt = 0;
    long long bofs = 0;
    static constexpr int kTileGran = 16;   // hand-off values per step: 8 plane-edge + 8 line-edge
    long long ngran() const { return tile ? (long long)nbands * T * kTileGran : (long long)nz * nbands * T; }
    long long slot(long long r) const {
        if (r < bnt) return r;
        return bofs + grid_slot(r - bnt);
    }
    long long grid_slot(long long r) const {
        const long long nxy = (long long)nx * ny;
        const long long k = r / nxy, q = r % nxy;
        if (tile) {
            const int j = (int)(q / nx), i = (int)(q % nx), a = j & 7, c = (int)(k & 7);
            const int l = a + 8 * (c ^ (c >> 1)), t = i + a + c;
            const long long band = (k >> 3) * NJ + (j >> 3);
            return ((band * (T / 2) + t / 2) * 64 + l) * 2 + (t & 1);
        }
        const int j = (int)(q / nx), i = (int)(q % nx), l = j & 63, t = i + skew * l + (skew - 1);
        return k * P2 + ((((long long)(j >> 6) * (T / 2) + t / 2) * 64 + l) * 2 + (t & 1));
    }
};
// detect: L off-diagonals only at offsets {nx, nx-1, .., nx-k, 1} in this order
// and U at {nx, nx-1, .., nx-k, 1} (canonical orders; k <= 2: ILU(0..2) of a
// 5-point grid), no wrap-around entries; skew = k + 1.  ok=false otherwise.
// split_u: U rows at {1, nx} in this order instead (ascending columns, the
// split U factor of MyILUPP::HostPrecond_right, src/preconditioner.cu:1117-1137),
// no fill (k = 0); sets u_inline_first.
Wave2D detect_wave2d(const CanonTri &L, const CanonTri &U, bool split_u = false);
// 3D: offsets {nx*ny, nx, 1} in this order in L and in U (canonical orders),
// no wrap-around; nz >= 2 planes of the 2D layout
Wave2D detect_wave3d(const CanonTri &L, const CanonTri &U);
// Bordered 2D grid: rows [0, nt) a small tail (any pattern), rows [nt, n) an
// unskewed 5-point grid block that detect_wave2d accepts once the tail columns
// are stripped from its L rows (they must lead each row's canonical order: the
// tail is solved first, and b - sum(tail terms) is the head of the row's own
// sum).  U rows of the grid reference the grid only (U rows of the tail may
// reference anything).  gl / gu: the grid block's triangles (indices - nt, tail
// terms of L stripped).  ok=false otherwise.
Wave2D detect_border2d(const CanonTri &L, const CanonTri &U, bool split_u, CanonTri &gl, CanonTri &gu);
// the split engine's layout choice (gg_set_precond_split, gg_host_split_layout):
// the 2D wavefront, else the bordered grid, honouring GG_NO_WAVEFRONT=1 (flow
// kernel for everything) and GG_NO_BORDER=1 (no bordered grid); at most 512 bands
Wave2D select_split_layout(const CanonTri &L, const CanonTri &U, CanonTri &gl, CanonTri &gu);

// rows with more off-diagonal terms than this are solved by a whole wave in the
// sync-free triangular solve (kernels.hip k_trsv_flow)
constexpr int kFlowLong = 32;
// bordered-grid tails this small run in one workgroup (kernels.hip k_tail_small)
constexpr int kTailSmallRows = 16384, kTailSmallLevels = 256;

// SpMV row blocks: each block <= 256 rows and <= kSpmvCap nnz (CSR-stream)
constexpr int kSpmvCap = 2048;
std::vector<int> spmv_blocks(const Csr &A, std::vector<int> &long_rows);

// ----------------------------------------------------------- device buffers
template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        release();
        if (count == 0) count = 1;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            throw Error{GG_ENOMEM, "hipMalloc(" + std::to_string(count * sizeof(T)) + " B) failed"};
        }
        n = count;
    }
    void upload(const T *h, size_t count, hipStream_t st) {
        alloc(count);
        if (count) GG_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, st));
    }
    void upload(const std::vector<T> &h, hipStream_t st) { upload(h.data(), h.size(), st); }
};

struct DevCsr {
    int n = 0, nnz = 0;
    DBuf<int> rp, ci;
    DBuf<double> v;
    // CSR-stream partition
    int nblk = 0;
    DBuf<int> blk;           // nblk+1 row boundaries
    int nlong = 0;
    DBuf<int> long_rows;     // rows too long for one block (vector-per-row path)
    // sliced ELL (one 64-row slice per wave, entry k of the slice's lane l at
    // sptr[s] + 64 k + l, padding col -1), used when rows are short and even
    bool sell = false;
    int nslice = 0;
    DBuf<int> sptr, sci;
    DBuf<double> sv;
    // column panels (k_spmv_panel; large matrices with scattered columns and
    // rows in ascending column order, GG_SPMV_PANEL): x cut into npanel panels
    // of pw entries, small enough for an XCD's L2; per panel its row segments
    // (seg_row: the row, ~row for a row's first segment; seg_ptr: the
    // segment's entries in the panel-major copy pci / pv), pan_seg[p] the
    // panel's first segment.  Panel by panel, a row's terms are added into its
    // running sum kept in y -- the CSR order, so the same bits
    bool panel = false;
    int npanel = 0, pw = 0;
    long long nseg = 0;
    DBuf<int> pan_seg, seg_row, seg_ptr, pci, zero_rows;
    // k_spmv_panel's blocks: per panel runs of <= 256 segments / <= kSpmvCap
    // entries, pblk = their first segments (panel p's blocks at pan_blk_h[p])
    DBuf<int> pblk;
    std::vector<int> pan_blk_h;
    DBuf<double> pv;
    int nzero = 0;
    // row tiles (k_spmv_rtile, GG_SPMV_RTILE): ONE launch of rtile blocks, block
    // b owning a contiguous row range and walking its sub-blocks rt_sub[b] ..
    // rt_sub[b+1]-1 (pblk indices) panel by panel; a segment longer than a
    // sub-block's capacity is cut into consecutive pieces (seg_row >= 0 after
    // the first).  0: the panel-major launches above
    int rtile = 0;
    DBuf<int> rt_sub;
    void upload(const Csr &A, hipStream_t st);
    void build_panels(const Csr &A, hipStream_t st);   // (upload: the column panels when they apply)
    void copy_from(const DevCsr &o, hipStream_t st);   // device-side duplicate
};

// wavefront division modes: unit diagonal, IEEE division, reciprocal + FMA
// corrections (both RN(acc/d)), multiply by the reciprocal (gg_set_division
// GG_DIV_RCP: RN(acc * RN(1/d)), tolerance parity); gg_set_division GG_DIV_FMA
// on an unskewed 2D grid: the row as two fused multiply-adds, in-line term
// first -- unit (WD_UFMA) or with the coefficients and b pre-scaled by RN(1/d)
// (WD_SFMA), tolerance parity
enum WaveDiv { WD_UNIT = 0, WD_HW = 1, WD_RCP = 2, WD_MUL = 3, WD_UFMA = 4, WD_SFMA = 5 };

// device triangular solve
struct DevTri {
    enum Kind { NONE, LEVEL, WAVE2D } kind = NONE;
    bool lower = true;
    int n = 0;
    // LEVEL
    DevCsr off;
    DBuf<double> d;
    std::vector<int> lev_ptr;    // host
    DBuf<int> lev_rows;
    DBuf<int> lev_ptr_d;         // a small bordered tail (k_tail_small): lev_ptr on the device
    // the flow kernel's tasks over lev_rows (level order): {first, count} = up
    // to 64 rows of at most kFlowLong terms, one per lane; count = -1: one row
    // with more terms, taken by a whole wave; {.z, .w} = the run's first
    // 64-entry group and width in the sliced copy (ell)
    int ntask = 0;
    DBuf<int4> tasks;
    // sliced (ELL) copy of the short rows' terms, per task w groups of 64
    // entries, group k = every lane's k-th term (canonical order; column -1
    // past a row's end): the kernel reads a lane's terms without rp and with
    // one coalesced load per term index (k_trsv_flow<true>)
    bool ell = false;
    DBuf<int> eci;
    DBuf<double> ev;
    // WAVE2D (layout arrays, length P)
    Wave2D wl;
    DBuf<double> c1, c2, dw, rw; // c1: |offset|=nx coef, c2: |offset|=1 coef, dw: divisor, rw: RN(1/dw)
    DBuf<double> c1s, c2s, c0s;  // WD_SFMA: RN(c1 * rw), RN(c2 * rw) (3D tiles: RN(c0 * rw))
    DBuf<double> ce1s, ce2s;     // WD_SFMA on a skewed grid: the fill coefficients pre-scaled too
    DBuf<double> c0;             // 3D: |offset| = nx*ny coefficient
    DBuf<double> ce1, ce2;       // skew 2/3 (ILU(1)/(2) fill): |offset| = nx-1, nx-2 coefficients
    DBuf<unsigned long long> prog;   // 3D: per (plane, band) batches stored (0 between launches)
    DBuf<int> order;             // 3D tiles: forward dependency order (the backward solve reverses it)
    bool il = false;             // upper 2D: in-line term first (Wave2D::u_inline_first)
    int div = WD_UNIT;           // division mode (kernels.hip k_trsv_wave2d)
    bool rcp_ok = false;         // every divisor admits WD_RCP
    bool mul_ok = false;         // every 1/d is finite and normal (WD_MUL admissible; rw uploaded)
    bool fma_ok = false;         // unskewed 2D grid / 3D tiles, canonical order, unit L or mul_ok U (c*s uploaded)
    int fast = 0;                // the owner's gg_set_division mode (GG_DIV_RCP: WD_MUL, GG_DIV_FMA: WD_*FMA)
    bool prefilled = false;      // LEVEL, per launch: x already holds the sentinel (flow kernel)
    bool mul = false;            // LEVEL, per launch: x = RN(acc * rw) (a bordered grid's tail under WD_MUL)
    bool fmrow = false;          // LEVEL: GG_DIV_FMA's rows (terms pre-scaled, fused order; rw = RN(1/d) or none)
    bool tile_queue = false;     // 3D tiles: claim tiles from a queue (after a non-resident static grid)
    int eff_div() const
    {
        if (fast == 2 && fma_ok) return div == WD_UNIT ? (int)WD_UFMA : (int)WD_SFMA;
        return (fast && mul_ok && div != WD_UNIT) ? (int)WD_MUL : div;
    }
    DBuf<unsigned long long> bnd;  // nbands * T hand-off granules (sentinel = not ready) + 128 dummies
    DBuf<unsigned long long> fcnt; // fused SpMV (forward solve): per slice group, 1 = stored (0 between launches)
    long long *trace = nullptr;  // diagnostics: per band, nbatch+1 timestamps (gg_trace_precond)
    double bytes = 0;            // algorithmic bytes per solve
    double bytes_mul = 0;        // the same with WD_MUL (y streamed in place of d (, y))
    // WAVE2D: what the kernel streams (no index arrays; bytes above = SURVEY.md
    // 8(d)'s CSR formulation), 0 = the same as bytes
    double stream_bytes = 0, stream_bytes_mul = 0;
    double alg_bytes() const
    {
        const int e = eff_div();
        return ((e == WD_MUL || e == WD_SFMA) ? bytes_mul : bytes) + (tail ? tail->bytes + cbytes : 0.0);
    }
    double stream_alg_bytes() const
    {
        const int e = eff_div();
        const double own = (e == WD_MUL || e == WD_SFMA) ? (stream_bytes_mul > 0 ? stream_bytes_mul : bytes_mul)
                                                         : (stream_bytes > 0 ? stream_bytes : bytes);
        return own + (tail ? tail->bytes + cbytes : 0.0);
    }
    // Bordered grid (Wave2D::bnt; this triangle = the grid block's wavefront,
    // its arrays and pointers relative to slot bofs): the tail rows as a LEVEL
    // triangle over the whole layout (columns are slots), solved by the flow
    // kernel before the grid (lower) or after it (upper); the lower grid rows'
    // tail terms as a coupling CSR (absolute row slots, tail columns) applied to
    // b in place between the two (b must be scratch: the split engine's t1)
    std::unique_ptr<DevTri> tail;
    std::unique_ptr<DevTri> tail_fma;   // the same rows as GG_DIV_FMA forms them (when fma_ok)
    long long bofs = 0;
    int ncoup = 0;
    DBuf<long long> cslot;
    DBuf<int> crp, cci;
    DBuf<double> cv;
    double cbytes = 0;
};

// device triangle from a canonical one: WAVE2D when `wl` is an active grid
// layout (nat2lay: row -> slot, arrays of length Ppad), else LEVEL (solver.hip)
void build_tri(DevTri &T, const CanonTri &C, const Wave2D *wl, const std::vector<long long> *nat2lay,
               long long Ppad, hipStream_t st);
// bordered grid (wl.bnt > 0): C the whole canonical triangle, Cg its grid
// block (detect_border2d); exact division only (the tail's flow kernel divides)
void build_tri_bordered(DevTri &T, const CanonTri &C, const CanonTri &Cg, const Wave2D &wl, hipStream_t st);
long long round_up(long long a, long long b);

struct DevState;   // device-side GMRES control block (kernels.h)

}  // namespace gg
