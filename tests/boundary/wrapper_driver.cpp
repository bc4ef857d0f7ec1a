// wrapper_driver.cpp -- a stand-in for a caller of the legacy GPU transient
// wrapper (src/gpuData.h:218-223; the reference's call site is
// src/mna_solve_gpu_gmres.cpp:755-756), compiled with g++ against libggmres.so:
// it builds the cs_dl matrices (CSC, long indices) and the gpuETBR block the
// way etbr's preparation does, calls wrapperGMRESforPG, and writes the port
// waveforms it returns.
//
//   wrapper_driver IN OUT
// IN  (little-endian): int32 n, nVS, nIS, numPts, nport, is_kind (0 none,
//     1 PWL, 2 PULSE, 3 both: the PWL block, then the PULSE block), use_single,
//     use_double; double tstep; then the CSC
//     matrices left, right, G, B, each int64 m, ncol, nnz, p[ncol+1], i[nnz],
//     double x[nnz]; int32 invPort[nport]; double dcVt[nVS]; PWL: int32
//     numPts[nIS], double time[nIS*64], value[nIS*64]; PULSE: double
//     time[nIS*5], value[nIS*2]
// OUT float x_single_host[numPts*nport], double x_host[numPts*nport]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gpuData.h"

namespace {

FILE *g_in;

template <class T>
std::vector<T> rd(size_t count)
{
    std::vector<T> v(count);
    if (count && std::fread(v.data(), sizeof(T), count, g_in) != count) {
        std::fprintf(stderr, "wrapper_driver: short input\n");
        std::exit(2);
    }
    return v;
}

struct Csc {
    std::vector<long> p, i;
    std::vector<double> x;
    ucr_cs_dl M{};
};

void read_csc(Csc &c)
{
    const std::vector<long> h = rd<long>(3);
    c.p = rd<long>(h[1] + 1);
    c.i = rd<long>(h[2]);
    c.x = rd<double>(h[2]);
    if (c.i.empty()) c.i.push_back(0);
    if (c.x.empty()) c.x.push_back(0.0);
    c.M.shallowCpy(h[2], h[0], h[1], c.p.data(), c.i.data(), c.x.data(), -1);   // nz == -1: compressed
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: wrapper_driver IN OUT\n");
        return 2;
    }
    g_in = std::fopen(argv[1], "rb");
    FILE *out = std::fopen(argv[2], "wb");
    if (!g_in || !out) return 2;
    const std::vector<int> hdr = rd<int>(8);
    const int n = hdr[0], nVS = hdr[1], nIS = hdr[2], numPts = hdr[3], nport = hdr[4], kind = hdr[5];
    gpuETBR e{};
    e.numPts = numPts;
    e.n = n;
    e.m = nVS + nIS;
    e.nport = nport;
    e.nVS = nVS;
    e.nIS = nIS;
    e.use_cuda_single = hdr[6];
    e.use_cuda_double = hdr[7];
    e.tstep = rd<double>(1)[0];
    e.tstop = e.tstep * (numPts - 1);
    Csc left, right, G, B;
    for (Csc *c : {&left, &right, &G, &B}) read_csc(*c);
    std::vector<int> port = rd<int>(nport);
    std::vector<double> dc = rd<double>(nVS);
    e.dcVt_host = dc.data();
    std::vector<int> pwl_n;
    std::vector<double> pwl_t, pwl_v, pul_t, pul_v;
    if (kind == 1 || kind == 3) {
        e.PWLcurExist = 1;
        pwl_n = rd<int>(nIS);
        pwl_t = rd<double>((size_t)nIS * MAX_PWL_PTS);
        pwl_v = rd<double>((size_t)nIS * MAX_PWL_PTS);
        e.PWLnumPts_host = pwl_n.data();
        e.PWLtime_host = pwl_t.data();
        e.PWLval_host = pwl_v.data();
    }
    if (kind == 2 || kind == 3) {
        e.PULSEcurExist = 1;
        pul_t = rd<double>((size_t)nIS * 5);
        pul_v = rd<double>((size_t)nIS * 2);
        e.PULSEtime_host = pul_t.data();
        e.PULSEval_host = pul_v.data();
    }
    std::vector<float> xs((size_t)numPts * nport, -1.0f);
    std::vector<double> xd((size_t)numPts * nport, -1.0);
    e.x_single_host = xs.data();
    e.x_host = xd.data();
    wrapperGMRESforPG(&left.M, &right.M, &G.M, &B.M, port.data(), nport, &e);
    std::fwrite(xs.data(), sizeof(float), xs.size(), out);
    std::fwrite(xd.data(), sizeof(double), xd.size(), out);
    std::fclose(out);
    std::fclose(g_in);
    return 0;
}
