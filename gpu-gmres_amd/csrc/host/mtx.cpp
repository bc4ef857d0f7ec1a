// mtx.cpp -- Matrix Market input: readSparseMatrix,
// src_thermal/SpMV_gen.cpp:93-187.  The reference skips '%' lines, reads
// "rows cols nnz" and nnz "row col value" triplets (all through %f, so indices
// written as floats are accepted and truncated), makes them 0-based and sorts
// them row-major (cmpRow: row, then column; :20-26).  Here: the same, with
// fp64 values, a stable sort (duplicates stay in file order), empty rows
// allowed, 'pattern' files valued 1, and optional expansion of symmetric /
// skew-symmetric files (the reference reads every file as general).
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../gg_internal.h"

namespace gg {

namespace {

std::string lower(std::string s)
{
    for (char &c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

struct Trip {
    int r, c;
    double v;
};

}  // namespace

bool read_mtx(const char *path, bool expand_symmetric, int &nrows, int &ncols, Csr &A)
{
    FILE *f = std::fopen(path, "r");
    if (!f) return false;
    char line[4096];
    bool pattern = false, symmetric = false, skew = false, complex_field = false;
    bool have_size = false;
    long long nnz = 0;
    while (std::fgets(line, sizeof line, f)) {
        if (line[0] == '%') {
            std::string l = lower(line);
            if (l.rfind("%%matrixmarket", 0) == 0) {
                pattern = l.find(" pattern") != std::string::npos;
                complex_field = l.find(" complex") != std::string::npos;
                skew = l.find("skew-symmetric") != std::string::npos;
                symmetric = !skew && (l.find(" symmetric") != std::string::npos ||
                                      l.find(" hermitian") != std::string::npos);
            }
            continue;
        }
        double a, b, c;
        if (std::sscanf(line, "%lf %lf %lf", &a, &b, &c) == 3) {
            nrows = (int)a;
            ncols = (int)b;
            nnz = (long long)c;
            have_size = true;
        }
        break;
    }
    if (!have_size || complex_field || nrows < 0 || ncols < 0 || nnz < 0) {
        std::fclose(f);
        return false;
    }
    std::vector<Trip> t;
    t.reserve((size_t)nnz * (expand_symmetric && (symmetric || skew) ? 2 : 1));
    for (long long i = 0; i < nnz; i++) {
        double r, c, v = 1.0;
        const int got = pattern ? std::fscanf(f, "%lf %lf", &r, &c) : std::fscanf(f, "%lf %lf %lf", &r, &c, &v);
        if (got != (pattern ? 2 : 3)) {
            std::fclose(f);
            return false;
        }
        const int ri = (int)r - 1, cj = (int)c - 1;       // 1-based in the file
        if (ri < 0 || ri >= nrows || cj < 0 || cj >= ncols) {
            std::fclose(f);
            return false;
        }
        t.push_back({ri, cj, v});
        if (expand_symmetric && (symmetric || skew) && ri != cj) t.push_back({cj, ri, skew ? -v : v});
    }
    std::fclose(f);
    std::stable_sort(t.begin(), t.end(),
                     [](const Trip &x, const Trip &y) { return x.r != y.r ? x.r < y.r : x.c < y.c; });
    A.n = nrows;
    A.rp.assign(nrows + 1, 0);
    A.ci.resize(t.size());
    A.v.resize(t.size());
    for (size_t k = 0; k < t.size(); k++) {
        A.rp[t[k].r + 1]++;
        A.ci[k] = t[k].c;
        A.v[k] = t[k].v;
    }
    for (int r = 0; r < nrows; r++) A.rp[r + 1] += A.rp[r];
    return true;
}

}  // namespace gg
