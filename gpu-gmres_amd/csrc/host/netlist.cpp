// SPICE power-grid netlist -> MNA system (G, C, B, source waveforms): the
// flat-netlist front end of the reference's transient path, restated:
//   node numbering   parser()            src/parser.cpp:69-272 (first pass;
//                    NodeList::findorPushNode, src/element.cpp:95-130)
//   G                stampG()            src/parser.cpp:1904-2099
//   C                stampC()            src/parser.cpp:2100-2268
//   B + waveforms    stampB()            src/parser.cpp:2269-2886
//   number suffixes  StrToNum()          src/parser.cpp:30-67
//   duplicates       matrix::pushEntry   src/matrix.cpp:91-130 (summed in push order)
// Host code only; the result feeds gg_set_matrix (A = G + C/h) and
// gg_transient_src.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "gg_internal.h"
#include "ggmres.h"
#include "ggmres_host.h"

namespace {

// StrToNum: strtod, then the SPICE scale suffix (only its first letter counts,
// "meg"/"MEG" -> 1e6; 'm' otherwise milli)
double str_to_num(const std::string &s)
{
    const char *p = s.c_str();
    char *end = nullptr;
    const double v = std::strtod(p, &end);
    switch (end[0]) {
    case 'T': case 't': return v * std::pow(10.0, 12);
    case 'G': case 'g': return v * std::pow(10.0, 9);
    case 'K': case 'k': return v * std::pow(10.0, 3);
    case 'M': case 'm':
        if (end[1] == 'E' || end[1] == 'e') return v * std::pow(10.0, 6);
        return v * std::pow(10.0, -3);
    case 'U': case 'u': return v * std::pow(10.0, -6);
    case 'n': case 'N': return v * std::pow(10.0, -9);
    case 'p': case 'P': return v * std::pow(10.0, -12);
    case 'f': case 'F': return v * std::pow(10.0, -15);
    default: return v;
    }
}

std::vector<std::string> tokens(const std::string &l)
{
    std::vector<std::string> t;
    std::istringstream is(l);
    std::string w;
    while (is >> w) t.push_back(w);
    return t;
}

// lines of the file with one level of .include inlined where it appears (the
// reference switches to the included file and back, src/parser.cpp:208-235)
bool read_lines(const std::string &path, std::vector<std::string> &out, int depth)
{
    std::ifstream f(path);
    if (!f) return false;
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "" : path.substr(0, slash + 1);
    std::string l;
    while (std::getline(f, l)) {
        if (!l.empty() && l.back() == '\r') l.pop_back();
        if (depth == 0 && l.size() > 2 && l[0] == '.' && l[1] == 'i' && l[2] == 'n') {
            std::vector<std::string> t = tokens(l);
            if (t.size() >= 2) {
                std::string inc;
                for (char c : t[1])
                    if (c != '"') inc += c;
                if (!read_lines(dir + inc, out, 1)) return false;
                continue;
            }
        }
        out.push_back(l);
    }
    return true;
}

struct Trip {
    int i, j;
    long long seq;
    double v;
};

struct Builder {
    std::vector<Trip> t;
    void push(int i, int j, double v) { t.push_back({i, j, (long long)t.size(), v}); }
    // CSR, columns ascending, duplicates summed in push order
    void csr(int nrows, int **rp, int **ci, double **val)
    {
        std::sort(t.begin(), t.end(), [](const Trip &a, const Trip &b) {
            return a.i != b.i ? a.i < b.i : a.j != b.j ? a.j < b.j : a.seq < b.seq;
        });
        std::vector<int> r(nrows + 1, 0), c;
        std::vector<double> v;
        for (size_t k = 0; k < t.size();) {
            size_t e = k;
            double s = t[k].v;
            while (++e < t.size() && t[e].i == t[k].i && t[e].j == t[k].j) s += t[e].v;
            c.push_back(t[k].j);
            v.push_back(s);
            r[t[k].i + 1]++;
            k = e;
        }
        for (int q = 0; q < nrows; q++) r[q + 1] += r[q];
        *rp = (int *)std::malloc(sizeof(int) * (nrows + 1));
        *ci = (int *)std::malloc(sizeof(int) * std::max<size_t>(c.size(), 1));
        *val = (double *)std::malloc(sizeof(double) * std::max<size_t>(v.size(), 1));
        std::copy(r.begin(), r.end(), *rp);
        std::copy(c.begin(), c.end(), *ci);
        std::copy(v.begin(), v.end(), *val);
    }
};

struct Src {
    int kind = GG_SRC_DC;
    std::vector<double> data;
};

// PWL points from the text between '(' and ')' of the element line: time/value
// pairs separated by blanks; a first point at t != 0 is preceded by (0, v)
void pwl_points(const std::string &line, Src &s)
{
    const size_t a = line.find('('), b = line.find(')', a == std::string::npos ? 0 : a);
    if (a == std::string::npos) return;
    std::vector<std::string> t = tokens(line.substr(a + 1, (b == std::string::npos ? line.size() : b) - a - 1));
    for (size_t k = 0; k + 1 < t.size(); k += 2) {
        const double tm = str_to_num(t[k]), v = str_to_num(t[k + 1]);
        if (s.data.empty() && tm != 0.0) {
            s.data.push_back(0.0);
            s.data.push_back(v);
        }
        s.data.push_back(tm);
        s.data.push_back(v);
    }
}

// PULSE(v1, v2, td, tr, tf, pw, period): the numbers between the '(' after the
// keyword and the next ')', separated by blanks and/or commas.  On the
// reference's own spelling ("PULSE(v1, v2, ..., period)") this reads the same
// values as its fixed-offset sscanf (src/parser.cpp:2655-2686); a blank
// before '(' or after it is accepted too.  Fewer than 7 numbers: empty.
std::vector<double> pulse_args(const std::string &line, size_t kw)
{
    const size_t a = line.find('(', kw);
    if (a == std::string::npos) return {};
    const size_t b = line.find(')', a);
    std::string body = line.substr(a + 1, (b == std::string::npos ? line.size() : b) - a - 1);
    for (char &ch : body)
        if (ch == ',') ch = ' ';
    std::vector<std::string> t = tokens(body);
    if (t.size() < 7) return {};
    std::vector<double> v;
    for (int k = 0; k < 7; k++) v.push_back(str_to_num(t[k]));
    return v;
}

// an element line R/C/L/V/I needs its name, two nodes and a value: both
// passes apply the same rule, and a shorter line rejects the netlist (naming
// it) instead of reserving an unknown it never stamps
void check_element(const std::vector<std::string> &t, const std::string &l)
{
    if (t.size() < 4)
        throw gg::Error{GG_EINVAL, "netlist: element line needs a name, two nodes and a value: '" + l + "'"};
}

}  // namespace

extern "C" int gg_host_read_netlist(const char *path, gg_netlist *out)
{
    if (!path || !out) return GG_EINVAL;
    std::memset(out, 0, sizeof(*out));
    std::vector<std::string> lines;
    if (!read_lines(path, lines, 0)) return GG_EINVAL;
    try {
        // ---- pass 1 (parser): node rows by first appearance, element counts, .tran, ports
        std::map<std::string, int> row;       // name -> row (-1 = ground)
        int nnodes = 0, nl = 0, nv = 0, ni = 0;
        double tstep = 0.0, tstop = 0.0;
        std::vector<std::string> ports;
        auto node = [&](const std::string &nm) {
            auto it = row.find(nm);
            if (it != row.end()) return it->second;
            const int r = (nm == "0" || nm == "gnd") ? -1 : nnodes++;
            row[nm] = r;
            return r;
        };
        for (const std::string &l : lines) {
            if (l.empty()) continue;
            const char c = (char)std::toupper((unsigned char)l[0]);
            if (c == 'R' || c == 'C' || c == 'L' || c == 'V' || c == 'I') {
                std::vector<std::string> t = tokens(l);
                check_element(t, l);
                if (c == 'L') nl++;
                if (c == 'V') nv++;
                if (c == 'I') ni++;
                node(t[1]);
                node(t[2]);
            } else if (c == '.' && l.size() > 1) {
                if (l[1] == 't') {
                    std::vector<std::string> t = tokens(l);
                    if (t.size() >= 3) {
                        tstep = str_to_num(t[1]);
                        tstop = str_to_num(t[2]);
                    }
                } else if (l.size() > 2 && l[1] == 'p' && l[2] == 'r') {
                    for (size_t k = 0; k < l.size(); k++)
                        if (l[k] == '(') {
                            const size_t e = l.find(')', k);
                            if (e == std::string::npos) break;
                            ports.push_back(l.substr(k + 1, e - k - 1));
                            k = e;
                        }
                }
            }
        }
        const int n = nnodes + nl + nv, nsrc = nv + ni;
        // ---- pass 2 (stampG, stampC, stampB: one pass in file order; each
        // matrix sees its own elements in the same order as its own pass)
        Builder G, Cm, B;
        std::vector<Src> src(nsrc);
        int il = 0, iv = -1, ii = -1;
        Src *last = nullptr;                  // the source '+' lines extend
        for (const std::string &l : lines) {
            if (l.empty()) continue;
            const char c = (char)std::toupper((unsigned char)l[0]);
            std::vector<std::string> t = tokens(l);
            if (c == '+') {
                // "%*2c %s %s": one (time, value) point per continuation line
                std::vector<std::string> p = tokens(l.size() > 2 ? l.substr(2) : std::string());
                if (last && p.size() >= 2) {
                    const double tm = str_to_num(p[0]), v = str_to_num(p[1]);
                    if (last->data.empty() && tm != 0.0) {
                        last->data.push_back(0.0);
                        last->data.push_back(v);
                    }
                    last->data.push_back(tm);
                    last->data.push_back(v);
                }
                continue;
            }
            if (!(c == 'R' || c == 'C' || c == 'L' || c == 'V' || c == 'I')) continue;
            check_element(t, l);
            if (c == 'V') iv++;
            if (c == 'I') ii++;
            const int n1 = row.at(t[1]), n2 = row.at(t[2]);
            if (c == 'R' || c == 'C') {
                const double v = c == 'R' ? 1.0 / str_to_num(t[3]) : str_to_num(t[3]);
                Builder &M = c == 'R' ? G : Cm;
                if (n1 >= 0) M.push(n1, n1, v);
                if (n2 >= 0) M.push(n2, n2, v);
                if (n1 >= 0 && n2 >= 0) {
                    M.push(n1, n2, -v);
                    M.push(n2, n1, -v);
                }
            } else if (c == 'L') {
                const int k = nnodes + il++;
                if (n1 >= 0) {
                    G.push(k, n1, -1.0);
                    G.push(n1, k, 1.0);
                }
                if (n2 >= 0) {
                    G.push(k, n2, 1.0);
                    G.push(n2, k, -1.0);
                }
                Cm.push(k, k, str_to_num(t[3]));
            } else {
                const int j = c == 'V' ? iv : nv + ii;
                if (c == 'V') {
                    const int k = nnodes + nl + iv;
                    if (n1 >= 0) {
                        G.push(n1, k, 1.0);
                        G.push(k, n1, -1.0);
                    }
                    if (n2 >= 0) {
                        G.push(n2, k, -1.0);
                        G.push(k, n2, 1.0);
                    }
                    B.push(k, j, -1.0);
                } else {
                    if (n1 >= 0) B.push(n1, j, -1.0);
                    if (n2 >= 0) B.push(n2, j, 1.0);
                }
                Src &s = src[j];
                last = &s;
                const std::string &w = t[3];
                const bool pw = w.size() >= 2 && (w[0] == 'P' || w[0] == 'p') && (w[1] == 'W' || w[1] == 'w');
                const bool pu = t.size() >= 5 && t[4].size() >= 2 && (t[4][0] == 'P' || t[4][0] == 'p') &&
                                (t[4][1] == 'U' || t[4][1] == 'u');
                if (pw) {
                    s.kind = GG_SRC_PWL;
                    pwl_points(l, s);
                } else if (pu) {
                    // "<dc> PULSE(v1, v2, td, tr, tf, pw, period)": the GPU path's
                    // gen_PULSEut_kernel parameters (the CPU path expands them to PWL)
                    s.kind = GG_SRC_PULSE;
                    s.data = pulse_args(l, l.find(t[4]));
                    if (s.data.empty()) {
                        s.kind = GG_SRC_DC;          // malformed: no waveform (value 0)
                        s.data = {0.0};
                    }
                } else {
                    s.kind = GG_SRC_DC;
                    s.data = {str_to_num(w)};
                }
            }
        }
        out->n_nodes = nnodes;
        out->n_l = nl;
        out->n_v = nv;
        out->n_i = ni;
        out->n = n;
        out->tstep = tstep;
        out->tstop = tstop;
        G.csr(n, &out->g_row_ptr, &out->g_col_idx, &out->g_val);
        Cm.csr(n, &out->c_row_ptr, &out->c_col_idx, &out->c_val);
        B.csr(n, &out->b_row_ptr, &out->b_col_idx, &out->b_val);
        out->src_kind = (int *)std::malloc(sizeof(int) * std::max(nsrc, 1));
        out->src_ptr = (int *)std::malloc(sizeof(int) * (nsrc + 1));
        size_t tot = 0;
        for (const Src &s : src) tot += s.data.size();
        out->src_data = (double *)std::malloc(sizeof(double) * std::max<size_t>(tot, 1));
        out->src_ptr[0] = 0;
        for (int k = 0; k < nsrc; k++) {
            out->src_kind[k] = src[k].kind;
            std::copy(src[k].data.begin(), src[k].data.end(), out->src_data + out->src_ptr[k]);
            out->src_ptr[k + 1] = out->src_ptr[k] + (int)src[k].data.size();
        }
        out->nport = (int)ports.size();
        out->port = (int *)std::malloc(sizeof(int) * std::max(out->nport, 1));
        for (int k = 0; k < out->nport; k++) {
            auto it = row.find(ports[k]);
            out->port[k] = it == row.end() ? -1 : it->second;
        }
    } catch (const gg::Error &e) {
        gg_host_free_netlist(out);
        gg::set_error(e.msg);
        return e.code;
    } catch (...) {
        gg_host_free_netlist(out);
        return GG_EINVAL;
    }
    return GG_OK;
}

extern "C" void gg_host_free_netlist(gg_netlist *nl)
{
    if (!nl) return;
    void *p[] = {nl->g_row_ptr, nl->g_col_idx, nl->g_val, nl->c_row_ptr, nl->c_col_idx, nl->c_val,
                 nl->b_row_ptr, nl->b_col_idx, nl->b_val, nl->src_kind, nl->src_ptr, nl->src_data, nl->port};
    for (void *q : p) std::free(q);
    std::memset(nl, 0, sizeof(*nl));
}
