// gmres_host.cpp -- the reference's HOST engine behind GMRES_host_PG: GMRESilu
// (src/gmres.cu:2069-2252) with the ILU++ split preconditioner's host applies
// (MyILUPP::HostPrecond_left / _right / _starting_value, src/preconditioner.cu:
// 1074-1137), restated in fp64 C++ as product code -- so a caller of
// gmresInterfacePG(float)::GMRES_host_PG (src/gmres_interface_pg.cu:62-108;
// mna_solve_gpu_gmres.cpp's CPU-only driver, :875, :1180) gets a CPU solve, as
// with the reference, not the device engine.
//
// Arithmetic: the reference's serial order everywhere (dots / norms summed
// serially from 0.0, src/gmres.cu:60-74; every row of the SpMV and the
// triangular solves in CSR order; a*b+c as two roundings -- the library is
// built with -ffp-contract=off).  The element-wise loops (SpMV rows, AXPYs,
// scalings, the update) run on a small pool of host threads: each element is
// computed exactly as in the serial loop, so the result is the same bits for
// any thread count; the dot products and the triangular solves stay serial, as
// in the reference.  Deviations shared with the device engine:
// fp64 instead of fp32; a cycle cut short by max_iter updates with its last
// filled column; a lucky breakdown (H[i+1,i] = 0) sets v_{i+1} = 0.
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "ggmres_host.h"
#include "gmres_host.h"

namespace gg {

namespace {

// ---- a fixed pool of host threads for the element-wise loops -------------------
class Pool {
   public:
    static Pool &get()
    {
        static Pool p;
        return p;
    }
    int size() const { return (int)th_.size() + 1; }
    // f(lo, hi) over [0, n) in size() contiguous chunks (the caller runs chunk 0)
    void run(long long n, const std::function<void(long long, long long)> &f)
    {
        const int T = size();
        if (T == 1 || n < kMinParallel) {
            f(0, n);
            return;
        }
        std::unique_lock<std::mutex> lk(m_);
        job_ = &f;
        n_ = n;
        pending_ = T - 1;
        gen_++;
        lk.unlock();
        cv_.notify_all();
        f(0, chunk(0, n, T).second);
        lk.lock();
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            gen_++;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
    }

   private:
    static constexpr long long kMinParallel = 1 << 15;
    static std::pair<long long, long long> chunk(int k, long long n, int T)
    {
        const long long q = n / T, r = n % T;
        const long long lo = k * q + std::min<long long>(k, r);
        return {lo, lo + q + (k < r ? 1 : 0)};
    }
    Pool()
    {
        int t = (int)std::thread::hardware_concurrency();
        const char *e = std::getenv("GG_HOST_THREADS");
        if (e && std::atoi(e) > 0) t = std::atoi(e);
        t = std::max(1, std::min(t, 16));
        for (int k = 1; k < t; k++) th_.emplace_back([this, k] { loop(k); });
    }
    void loop(int k)
    {
        unsigned long long seen = 0;
        while (true) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const std::function<void(long long, long long)> *f = job_;
            const long long n = n_;
            lk.unlock();
            const auto c = chunk(k, n, size());
            (*f)(c.first, c.second);
            lk.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(long long, long long)> *job_ = nullptr;
    long long n_ = 0;
    int pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

template <class F>
void par_for(long long n, F &&body)
{
    Pool::get().run(n, [&](long long lo, long long hi) {
        for (long long i = lo; i < hi; i++) body(i);
    });
}

// sgemv's y = alpha A x + beta y with alpha = -1, beta = 1 (src/gmres.cu:77-88),
// and the plain SpMV (computeSpMV, src/SpMV_compute.cpp:19-36): rows in CSR order
void spmv(const HostSplitEngine &E, const double *x, double *y)
{
    par_for(E.n, [&](long long i) {
        double t = 0.0;
        for (int j = E.arp[i]; j < E.arp[i + 1]; j++) t += E.av[j] * x[E.aci[j]];
        y[i] = t;
    });
}
void residual(const HostSplitEngine &E, const double *x, const double *b, double *r, std::vector<double> &t)
{
    spmv(E, x, t.data());
    par_for(E.n, [&](long long i) { r[i] = -1.0 * t[i] + 1.0 * b[i]; });
}

// HostPrecond_left (src/preconditioner.cu:1094-1114): t = in / lscale, gathered
// by perm_row, forward solve with L (diagonal last in each row)
void split_left(const HostSplitEngine &E, const double *in, double *out, std::vector<double> &t)
{
    const int n = E.n;
    par_for(n, [&](long long i) { t[i] = in[i] / E.ls[i]; });
    par_for(n, [&](long long i) { out[i] = t[E.prow[i]]; });
    for (int i = 0; i < n; i++) {
        const int lb = E.lrp[i], ub = E.lrp[i + 1];
        for (int j = lb; j < ub - 1; j++) out[i] -= E.lv[j] * out[E.lci[j]];
        out[i] = out[i] / E.lv[ub - 1];
    }
}
// HostPrecond_right (:1117-1137): t = in * middle, backward solve with U
// (diagonal first), scattered by perm_col and divided by rscale
void split_right(const HostSplitEngine &E, const double *in, double *out, std::vector<double> &t)
{
    const int n = E.n;
    par_for(n, [&](long long i) { t[i] = in[i] * E.mid[i]; });
    for (int i = n - 1; i >= 0; i--) {
        const int lb = E.urp[i], ub = E.urp[i + 1];
        for (int j = lb + 1; j < ub; j++) t[i] -= E.uv[j] * t[E.uci[j]];
        t[i] = t[i] / E.uv[lb];
    }
    par_for(n, [&](long long i) { out[i] = t[E.pcol[i]] / E.rs[i]; });
}
// HostPrecond_starting_value (:1074-1091): y = M^-1 U P_c^-1 D_r x
void split_start(const HostSplitEngine &E, const double *in, double *out, std::vector<double> &t,
                 std::vector<double> &z)
{
    const int n = E.n;
    par_for(n, [&](long long i) { t[i] = in[i] * E.rs[i]; });
    for (int i = 0; i < n; i++) z[E.pcol[i]] = t[i];
    par_for(n, [&](long long i) {
        double s = 0.0;
        for (int j = E.urp[i]; j < E.urp[i + 1]; j++) s += E.uv[j] * z[E.uci[j]];
        t[i] = s;
    });
    par_for(n, [&](long long i) { out[i] = t[i] / E.mid[i]; });
}

double dot(const double *x, const double *y, int n)
{
    double t = 0.0;                     // src/gmres.cu:68-74, serial
    for (int i = 0; i < n; i++) t += x[i] * y[i];
    return t;
}
double norm2(const double *v, int n)
{
    double t = 0.0;                     // src/gmres.cu:60-66, serial
    for (int i = 0; i < n; i++) t += v[i] * v[i];
    return std::sqrt(t);
}
void apply_rot(double &dx, double &dy, double cs, double sn)
{
    const double temp = cs * dx + sn * dy;     // ApplyPlaneRotation (src/gmres.cu:192-197)
    dy = -sn * dx + cs * dy;
    dx = temp;
}
void gen_rot(double dx, double dy, double &cs, double &sn)
{
    if (dy == 0.0) {                    // GeneratePlaneRotation (:200-216)
        cs = 1.0;
        sn = 0.0;
    } else if (std::fabs(dy) > std::fabs(dx)) {
        const double temp = dx / dy;
        sn = 1.0 / std::sqrt(1.0 + temp * temp);
        cs = temp * sn;
    } else {
        const double temp = dy / dx;
        cs = 1.0 / std::sqrt(1.0 + temp * temp);
        sn = temp * cs;
    }
}
// Update (src/gmres.cu:93-116): y = H(0:k,0:k)^-1 s by back substitution, then
// acc += sum_j V_j y_j in ascending j per element
void update(double *acc, int k, const std::vector<double> &H, int m, const std::vector<double> &s,
            const std::vector<double> &V, int n)
{
    std::vector<double> y(s.begin(), s.begin() + k + 1);
    for (int i = k; i >= 0; i--) {
        y[i] /= H[i + (size_t)i * (m + 1)];
        for (int j = i - 1; j >= 0; j--) y[j] -= H[j + (size_t)i * (m + 1)] * y[i];
    }
    par_for(n, [&](long long i) {
        double a = acc[i];
        for (int j = 0; j <= k; j++) a += V[(size_t)j * n + i] * y[j];
        acc[i] = a;
    });
}

}  // namespace

int host_threads() { return Pool::get().size(); }

int gmres_split_host(const HostSplitEngine &E, const double *b, double *x, int m, int *max_iter, double *tol,
                     int *inner_iters)
{
    const int n = E.n;
    const size_t nn = (size_t)std::max(n, 1);
    std::vector<double> s(m + 1, 0.0), cs(m + 1, 0.0), sn(m + 1, 0.0), H((size_t)(m + 1) * m, 0.0);
    std::vector<double> w(nn), ww(nn), r(nn), rr(nn), bb(nn), y(nn, 0.0), t(nn), z(nn);
    std::vector<double> V((size_t)(m + 1) * nn);
    int done = 0;
    if (inner_iters) *inner_iters = 0;

    split_left(E, b, bb.data(), t);                           // HostPrecond_rhs (:2096-2098)
    double normb = norm2(bb.data(), n);
    if (normb == 0.0) normb = 1.0;
    split_start(E, x, y.data(), t, z);                        // HostPrecond_starting_value (:2102)
    residual(E, x, b, rr.data(), t);                          // rr = b - A x (:2103)
    split_left(E, rr.data(), r.data(), t);                    // r = Ml rr
    double beta = norm2(r.data(), n);
    double resid = beta / normb;
    if (resid <= *tol) {                                      // "<=" (:2112)
        *tol = resid;
        *max_iter = 0;
        return 0;
    }
    int j = 1;
    while (j <= *max_iter) {
        const double inv = 1.0 / beta;
        par_for(n, [&](long long q) { V[q] = inv * r[q]; });
        std::fill(s.begin(), s.end(), 0.0);
        s[0] = beta;
        int i;
        for (i = 0; i < m && j <= *max_iter; i++, j++) {
            double *vi = V.data() + (size_t)i * nn;
            split_right(E, vi, w.data(), t);                  // w = Mr v_i (:2143)
            spmv(E, w.data(), ww.data());                     // ww = A w (:2144)
            split_left(E, ww.data(), w.data(), t);            // w = Ml ww (:2145)
            for (int k = 0; k <= i; k++) {                    // MGS (:2146-2150)
                const double *vk = V.data() + (size_t)k * nn;
                const double h = dot(w.data(), vk, n);
                H[k + (size_t)i * (m + 1)] = h;
                const double a = -h;
                par_for(n, [&](long long q) { w[q] = a * vk[q] + w[q]; });
            }
            const double hn = norm2(w.data(), n);
            H[(i + 1) + (size_t)i * (m + 1)] = hn;
            double *vn = V.data() + (size_t)(i + 1) * nn;
            if (hn != 0.0) {
                const double hinv = 1.0 / hn;
                par_for(n, [&](long long q) { vn[q] = hinv * w[q]; });
            } else {
                std::fill(vn, vn + n, 0.0);                   // lucky breakdown: no division by 0
            }
            for (int k = 0; k < i; k++)
                apply_rot(H[k + (size_t)i * (m + 1)], H[(k + 1) + (size_t)i * (m + 1)], cs[k], sn[k]);
            gen_rot(H[i + (size_t)i * (m + 1)], H[(i + 1) + (size_t)i * (m + 1)], cs[i], sn[i]);
            apply_rot(H[i + (size_t)i * (m + 1)], H[(i + 1) + (size_t)i * (m + 1)], cs[i], sn[i]);
            apply_rot(s[i], s[i + 1], cs[i], sn[i]);
            done++;
            resid = std::fabs(s[i + 1]) / normb;
            if (resid < *tol) {                               // "<" (:2170)
                update(y.data(), i, H, m, s, V, n);
                split_right(E, y.data(), x, t);               // x = Mr y (:2176)
                *tol = resid;
                *max_iter = j;
                if (inner_iters) *inner_iters = done;
                return 0;
            }
        }
        update(y.data(), i - 1, H, m, s, V, n);               // the last filled column
        split_right(E, y.data(), x, t);
        residual(E, x, b, rr.data(), t);
        split_left(E, rr.data(), r.data(), t);
        beta = norm2(r.data(), n);
        resid = beta / normb;
        if (resid < *tol) {
            *tol = resid;
            *max_iter = j;
            if (inner_iters) *inner_iters = done;
            return 0;
        }
    }
    *tol = resid;
    if (inner_iters) *inner_iters = done;
    return 1;
}

}  // namespace gg
