/*
 * compat/gpuData.h -- the reference's GPU transient data block and legacy
 * transient wrapper (src/gpuData.h:43-116, 218-223), layout-identical, so a
 * driver that fills gpuETBR and calls wrapperGMRESforPG links against
 * libggmres.so unchanged (C++ linkage, as the reference declares it).
 *
 *   gpuETBR             src/gpuData.h:43-116   (member order and types are ABI;
 *                       static_asserts on the offsets in
 *                       gpu-gmres_amd/csrc/compat/wrapper_pg.cpp)
 *   wrapperGMRESforPG   src/gpuData.h:218-223, defined at src/wrapperGMRESforPG.cu:19-715
 *
 * What wrapperGMRESforPG computes here (the reference's solves are commented
 * out, src/wrapperGMRESforPG.cu:422-459, so its loop only forms right-hand
 * sides; this implementation performs the solves that loop was written for):
 *   u_i   = source values at t = i * tstep, i = 0 .. numPts-1: nVS DC voltage
 *           sources (dcVt_host) first, then nIS current sources (PWL tables
 *           PWLnumPts/PWLtime/PWLval, or PULSE PULSEtime {td, tr, tf, tw, tp} /
 *           PULSEval {vlo, vhi}), gen_dcVt / gen_PWLut / gen_PULSEut semantics
 *   x_0   = G^-1 (B u_0)                      (the DC point, i == 0)
 *   x_i   = left^-1 (B u_i + right x_{i-1})   (backward Euler, left = G + C/h,
 *                                              right = C/h), warm start x_{i-1}
 *   x_single_host[i * nport + j] = x_i[invPort[j]]   (use_cuda_single, float)
 *   x_host[i * nport + j]        = the same in double (use_cuda_double; the
 *                                  reference's double branch exits)
 * Each system is solved with GMRES(32) + ILU(0), tol 1e-7, at most 10000
 * iterations (the PG interface's settings, src/gmres_interface_pg.cu:7,66).
 * The output arrays are the caller's (nport * numPts elements).
 * Current sources, per source k: PWL when PWLcurExist and PWLnumPts_host[k] > 0
 * (at most MAX_PWL_PTS points read), else PULSE when PULSEcurExist, else 0.
 * (Deviation: the reference evaluates all nIS as PWL and then, when
 * PULSEcurExist, overwrites all nIS with PULSE, src/wrapperGMRESforPG.cu:331-392.)
 * Errors (bad sizes or ports, allocation / factorization / solve failure): the
 * reference aborts (checkCudaErrors); here the message goes to stderr and every
 * requested output element (x_single_host / x_host) is set to NaN.  A system
 * that does not converge in 10000 iterations prints "Failed to converge." as
 * the reference does and keeps its last iterate.
 */
#ifndef GG_COMPAT_GPUDATA_H_
#define GG_COMPAT_GPUDATA_H_

#include "SpMV.h"
#include "format_convert.h"

#define MAX_PWL_PTS 64

typedef struct {
    int numPts;   /* time zero is counted */
    int n;
    int q;
    int m;        /* nVS + nIS */
    int nport;

    int use_cuda_single, use_cuda_double;

    double tstep, tstop;
    double *ut_host;

    int *ipiv_host;
    double *V_host;
    double *LV_host;
    double *L_hCG_host;
    double *U_hCG_host;
    double *hC_host;
    double *Br_host;
    double *xr0_host;
    double *x_host;

    float *V_single_host;
    float *LV_single_host;
    float *L_hCG_single_host;
    float *U_hCG_single_host;
    float *hC_single_host;
    float *Br_single_host;
    float *xr0_single_host;
    float *x_single_host;

    int ldUt;
    double *ut_dev;
    int *ipiv_dev;
    double *V_dev;
    double *LV_dev;
    double *L_hCG_dev;
    double *U_hCG_dev;
    double *hC_dev;
    double *Br_dev;
    double *xr_dev;
    double *x_dev;

    float *ut_single_dev;
    float *V_single_dev;
    float *LV_single_dev;
    float *L_hCG_single_dev;
    float *U_hCG_single_dev;
    float *hC_single_dev;
    float *Br_single_dev;
    float *xr_single_dev;
    float *x_single_dev;

    int nIS, nVS;
    double *dcVt_host, *dcVt_dev;
    float *dcVt_single_host, *dcVt_single_dev;
    int PWLvolExist, PWLcurExist, PULSEvolExist, PULSEcurExist;

    int *PWLnumPts_host, *PWLnumPts_dev;
    double *PWLtime_host, *PWLtime_dev;
    double *PWLval_host, *PWLval_dev;

    float *PWLtime_single_host, *PWLtime_single_dev;
    float *PWLval_single_host, *PWLval_single_dev;

    double *PULSEtime_host, *PULSEtime_dev;
    double *PULSEval_host, *PULSEval_dev;

    float *PULSEtime_single_host, *PULSEtime_single_dev;
    float *PULSEval_single_host, *PULSEval_single_dev;
} gpuETBR;

void wrapperGMRESforPG(ucr_cs_dl *left, ucr_cs_dl *right, ucr_cs_dl *G, ucr_cs_dl *B,
                       int *invPort, int nport, gpuETBR *myGPUetbr);

#endif /* GG_COMPAT_GPUDATA_H_ */
