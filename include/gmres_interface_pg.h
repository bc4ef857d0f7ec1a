/*
 * gmres_interface_pg.h -- drop-in replacement of the reference's PG solver
 * boundary (src/gmres_interface_pg.h:1-75).  Same classes, same public data
 * members in the same order (the layout is ABI: mna_solve_gpu_gmres.cpp writes
 * rhs_h / xgmres_h and reads max_it / tol directly), same mangled methods.
 * The methods are implemented by libggmres.so on top of the C ABI in
 * ggmres.h: fp32 in/out at this boundary, fp64 inside.
 *
 *   setPrecondPG   src/gmres_interface_pg.cu:9-60    -> gg_set_matrix + gg_set_precond_split
 *   GMRES_dev_PG   src/gmres_interface_pg.cu:110-139 -> gg_solve (restart 32, max_it 10000, tol 1e-7)
 *   GMRES_host_PG  src/gmres_interface_pg.cu:62-108  -> the host GMRESilu engine (CPU, fp64,
 *                                                       csrc/host/gmres_host.cpp)
 */
#ifndef _GMRES_INTERFACE_PG_H_
#define _GMRES_INTERFACE_PG_H_
#include "SpMV.h"

class gmresInterfacePG {
 public:
  ~gmresInterfacePG();

  int matrixSize;

  float *h_val;
  int *h_rowPtr;
  int *h_colIdx;

  float *x_h;
  float *x_d;

  float *xgmres_h;
  float *rhs_h;

  void *Precond;   /* opaque: the device solver and the host engine */

  int max_it; /* both input and output */
  float tol;

  void setPrecondPG(MySpMatrix *A,
                    MySpMatrixDouble *PrLeft, MySpMatrixDouble *PrRight,
                    MySpMatrix *PrMiddle_mySpM,
                    MySpMatrix *PrPermRow, MySpMatrix *PrPermCol,
                    MySpMatrixDouble *PrLscale, MySpMatrixDouble *PrRscale);
  int GMRES_host_PG();
};

class gmresInterfacePGfloat {
 public:
  ~gmresInterfacePGfloat();

  int matrixSize;
  int nnz;
  float *h_val;
  int *h_rowPtr;
  int *h_colIdx;

  float *d_val;
  int *d_rowPtr;
  int *d_colIdx;

  float *x_h;
  float *x_d;

  float *xgmres_h;
  float *rhs_h;

  float *xgmres_d;
  float *rhs_d;

  void *Precond;   /* opaque: the device solver and the host engine */

  int max_it; /* both input and output */
  float tol;

  void setPrecondPG(MySpMatrix *A,
                    MySpMatrixDouble *PrLeft, MySpMatrixDouble *PrRight,
                    MySpMatrix *PrMiddle_mySpM,
                    MySpMatrix *PrPermRow, MySpMatrix *PrPermCol,
                    MySpMatrix *PrLscale, MySpMatrix *PrRscale);
  int GMRES_host_PG();
  int GMRES_dev_PG();
};

#endif
