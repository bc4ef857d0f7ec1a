// partition.cpp -- domain decomposition setup on the host:
//
//   partition_arrow   partition4        src/partition3.cpp:122-194
//                     (METIS_PartGraphRecursive is not in the image: replaced by
//                     our own recursive BFS bisection, or contiguous index blocks)
//   arrow_permute     the symmetric permutation the DD solve runs on
//                     (pinv / q of partition4 applied to rows and columns)
//   csr_block         dd_form's block extraction (As, E, F, At)  src/form_dd.cpp:32-110
//
// All of it is integer work; tests/test_partition.py checks it against the
// restatement in oracle/partition.py.
#include <algorithm>
#include <numeric>
#include <set>

#include "../gg_internal.h"

namespace gg {

namespace {

// symmetrized adjacency of A's pattern without the diagonal (METIS node graph:
// xadj / adjncy, neighbours ascending)
void node_graph(const Csr &A, std::vector<int> &xadj, std::vector<int> &adj)
{
    const int n = A.n;
    std::vector<std::vector<int>> nb(n);
    for (int r = 0; r < n; r++)
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
            const int c = A.ci[k];
            if (c == r) continue;
            nb[r].push_back(c);
            nb[c].push_back(r);
        }
    xadj.assign(n + 1, 0);
    adj.clear();
    for (int r = 0; r < n; r++) {
        std::sort(nb[r].begin(), nb[r].end());
        nb[r].erase(std::unique(nb[r].begin(), nb[r].end()), nb[r].end());
        adj.insert(adj.end(), nb[r].begin(), nb[r].end());
        xadj[r + 1] = (int)adj.size();
    }
}

// BFS order of the vertices of `set` (mark[v] == tag) from `start`; components
// not reached are continued from their smallest vertex.  Neighbours in
// ascending order.  Returns the order; `last` = the last vertex of the first
// component (a far vertex, for the pseudo-peripheral search).
std::vector<int> bfs_order(const std::vector<int> &xadj, const std::vector<int> &adj,
                           const std::vector<int> &set, const std::vector<int> &mark, int tag,
                           int start, std::vector<int> &seen, int stamp, int *last)
{
    std::vector<int> order;
    order.reserve(set.size());
    size_t next_root = 0;
    int root = start;
    bool first = true;
    while (order.size() < set.size()) {
        if (!first) {
            while (seen[set[next_root]] == stamp) next_root++;
            root = set[next_root];
        }
        size_t head = order.size();
        order.push_back(root);
        seen[root] = stamp;
        while (head < order.size()) {
            const int v = order[head++];
            for (int p = xadj[v]; p < xadj[v + 1]; p++) {
                const int w = adj[p];
                if (mark[w] == tag && seen[w] != stamp) {
                    seen[w] = stamp;
                    order.push_back(w);
                }
            }
        }
        if (first && last) *last = order.back();
        first = false;
    }
    return order;
}

// recursive bisection of `set` (ascending vertex ids) into k parts numbered
// from p0: BFS from a pseudo-peripheral vertex (two sweeps from the smallest
// vertex), the first |set|*k1/k vertices of the order form the first half
void bisect(const std::vector<int> &xadj, const std::vector<int> &adj, std::vector<int> set, int k,
            int p0, std::vector<int> &part, std::vector<int> &mark, std::vector<int> &seen, int &tag,
            int &stamp)
{
    if (k <= 1 || set.size() <= 1) {
        for (int v : set) part[v] = p0;
        return;
    }
    const int my = ++tag;
    for (int v : set) mark[v] = my;
    int far = set[0];
    bfs_order(xadj, adj, set, mark, my, set[0], seen, ++stamp, &far);
    std::vector<int> order = bfs_order(xadj, adj, set, mark, my, far, seen, ++stamp, nullptr);
    const int k1 = k / 2;
    const size_t n1 = (size_t)((long long)set.size() * k1 / k);
    std::vector<int> a(order.begin(), order.begin() + n1), b(order.begin() + n1, order.end());
    std::sort(a.begin(), a.end());
    std::sort(b.begin(), b.end());
    bisect(xadj, adj, std::move(a), k1, p0, part, mark, seen, tag, stamp);
    bisect(xadj, adj, std::move(b), k - k1, p0 + k1, part, mark, seen, tag, stamp);
}

}  // namespace

void grid_blocks(const Csr &A, int nparts, GridBlocks &gb)
{
    // line length: the most frequent |offset| above 1 of the pattern (ties: the
    // smallest); plane size: the most frequent larger offset that is a multiple
    // of it, if it is frequent (>= n/8 entries: a 7-point 3D grid)
    const int n = A.n;
    gb = GridBlocks{};
    std::vector<int> cnt;
    for (int r = 0; r < n; r++)
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
            const int o = std::abs(A.ci[k] - r);
            if (o > 1 && o <= (1 << 24)) {
                if ((int)cnt.size() <= o) cnt.resize(o + 1, 0);
                cnt[o]++;
            }
        }
    int nx = 0;
    for (int o = 2; o < (int)cnt.size(); o++)
        if (cnt[o] > (nx ? cnt[nx] : 0)) nx = o;
    if (nx == 0 || n % nx != 0) return;
    long long nxy = 0;
    for (long long o = 2LL * nx; o < (long long)cnt.size(); o += nx)
        if (cnt[o] >= n / 8 && cnt[o] > (nxy ? cnt[nxy] : 0)) nxy = o;
    if (nxy && n % nxy == 0 && n / nxy >= 2) {
        gb.nx = nx;
        gb.ny = (int)(nxy / nx);
        gb.nz = (int)(n / nxy);
        // px <= py <= pz, the most cube-like factorization
        int best = -1;
        for (int a = 1; a <= nparts; a++) {
            if (nparts % a) continue;
            for (int b = a; b <= nparts / a; b++) {
                if ((nparts / a) % b) continue;
                const int c = nparts / a / b;
                if (c < b) continue;
                if (best < 0 || c - a < best) {
                    best = c - a;
                    gb.px = a;
                    gb.py = b;
                    gb.pz = c;
                }
            }
        }
    } else {
        gb.nx = nx;
        gb.ny = n / nx;
        gb.nz = 1;
        // px the largest divisor of nparts not above sqrt(nparts), py = nparts / px
        gb.px = 1;
        for (int d = 1; (long long)d * d <= nparts; d++)
            if (nparts % d == 0) gb.px = d;
        gb.py = nparts / gb.px;
        gb.pz = 1;
    }
    if (gb.px > gb.nx || gb.py > gb.ny || gb.pz > gb.nz) gb = GridBlocks{};
}

void partition_arrow(const Csr &A, int nparts, int method, std::vector<int> &node_part,
                     std::vector<int> &part_size, std::vector<int> &pinv, std::vector<int> &q)
{
    const int n = A.n;
    std::vector<int> xadj, adj;
    node_graph(A, xadj, adj);
    node_part.assign(n, 0);
    if ((method & 3) == GG_PART_BLOCKS) {
        // contiguous index ranges: strips / slabs of a natural-order grid
        for (int j = 0; j < n; j++) node_part[j] = (int)((long long)j * nparts / n);
    } else if ((method & 3) == GG_PART_GRID) {
        // px x py rectangles of a natural-order 2D grid, px x py x pz boxes
        // of a 3D one (grid_blocks): each interior stays a rectangle / box in
        // row-major order, a sub-grid whose wavefront chain is nx/px + ny/py
        // (+ nz/pz) rather than a slab's nx + ny/N (nx + ny + nz/N)
        GridBlocks gb;
        grid_blocks(A, nparts, gb);
        GG_REQUIRE(gb.nx > 0, GG_EINVAL, "GG_PART_GRID: the matrix is not a natural-order grid");
        const long long nxy = (long long)gb.nx * gb.ny;
        for (int j = 0; j < n; j++) {
            const long long i = j % gb.nx, y = (j / gb.nx) % gb.ny, z = j / nxy;
            const int bx = (int)(i * gb.px / gb.nx), by = (int)(y * gb.py / gb.ny), bz = (int)(z * gb.pz / gb.nz);
            node_part[j] = (bz * gb.py + by) * gb.px + bx;
        }
    } else {
        std::vector<int> all(n), mark(n, 0), seen(n, 0);
        std::iota(all.begin(), all.end(), 0);
        int tag = 0, stamp = 0;
        bisect(xadj, adj, std::move(all), nparts, 0, node_part, mark, seen, tag, stamp);
    }
    // partition4's adjustment (src/partition3.cpp:149-162): every endpoint of
    // a cut edge moves to the separator part `nparts`
    std::set<int> toplevel;
    for (int j = 0; j < n; j++)
        for (int p = xadj[j]; p < xadj[j + 1]; p++)
            if (node_part[adj[p]] != node_part[j]) {
                toplevel.insert(adj[p]);
                toplevel.insert(j);
            }
    for (int v : toplevel) node_part[v] = nparts;
    // sizes, then pinv / q: interiors 0..nparts-1, separator last, ascending
    // original index inside a part (:166-193)
    part_size.assign(nparts + 1, 0);
    for (int j = 0; j < n; j++) part_size[node_part[j]]++;
    std::vector<int> begin(nparts + 2, 0);
    for (int i = 0; i <= nparts; i++) begin[i + 1] = begin[i] + part_size[i];
    std::vector<int> cur(nparts + 1, 0);
    pinv.assign(n, 0);
    q.assign(n, 0);
    for (int j = 0; j < n; j++) {
        const int p = node_part[j];
        pinv[j] = begin[p] + cur[p];
        q[begin[p] + cur[p]] = j;
        cur[p]++;
    }
    if (method & GG_PART_COLOR_SEP) {
        // extension: the separator ordered by a greedy colouring of its own
        // graph (first fit, ascending index), then by index -- the separator's
        // triangles become a few levels instead of chains as long as its lines
        const int s0 = begin[nparts];
        std::vector<int> color(n, -1);
        int ncol = 0;
        for (int i = s0; i < n; i++) {
            const int v = q[i];
            std::vector<char> used(ncol + 1, 0);
            for (int p = xadj[v]; p < xadj[v + 1]; p++) {
                const int w = adj[p];
                if (node_part[w] == nparts && color[w] >= 0) used[color[w]] = 1;
            }
            int c = 0;
            while (used[c]) c++;
            color[v] = c;
            ncol = std::max(ncol, c + 1);
        }
        std::stable_sort(q.begin() + s0, q.end(), [&](int a, int b) { return color[a] < color[b]; });
        for (int i = s0; i < n; i++) pinv[q[i]] = i;
    }
}

Csr arrow_permute(const Csr &A, const std::vector<int> &pinv, const std::vector<int> &q)
{
    const int n = A.n;
    Csr B;
    B.n = n;
    B.rp.assign(n + 1, 0);
    B.ci.resize(A.rp[n]);
    B.v.resize(A.rp[n]);
    std::vector<std::pair<int, double>> row;
    for (int i = 0; i < n; i++) {
        const int r = q[i];
        row.clear();
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) row.push_back({pinv[A.ci[k]], A.v[k]});
        std::stable_sort(row.begin(), row.end(),
                         [](const std::pair<int, double> &a, const std::pair<int, double> &b) {
                             return a.first < b.first;
                         });
        const int o = B.rp[i];
        for (size_t t = 0; t < row.size(); t++) {
            B.ci[o + t] = row[t].first;
            B.v[o + t] = row[t].second;
        }
        B.rp[i + 1] = o + (int)row.size();
    }
    return B;
}

Csr csr_block(const Csr &A, int r0, int r1, int c0, int c1)
{
    Csr B;
    B.n = r1 - r0;
    B.rp.assign(B.n + 1, 0);
    for (int r = r0; r < r1; r++) {
        for (int k = A.rp[r]; k < A.rp[r + 1]; k++) {
            const int c = A.ci[k];
            if (c >= c0 && c < c1) {
                B.ci.push_back(c - c0);
                B.v.push_back(A.v[k]);
            }
        }
        B.rp[r - r0 + 1] = (int)B.ci.size();
    }
    return B;
}

}  // namespace gg
