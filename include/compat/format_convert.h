/*
 * compat/format_convert.h -- the reference's boundary feed:
 * the CSC (long indices, double values) to CSR conversions its drivers run
 * before they hand matrices to the solver classes, with the reference's
 * semantics and C++ signatures (src/gpuData.h:144-209, src/formatConvert.cpp).
 *
 *   ucr_cs_dl                      src/gpuData.h:146-164 (layout-identical)
 *   coo2csr_in / coo2csrDouble_in  src/formatConvert.cpp:112-216 (in place,
 *                                  rows then a bubble sort by column)
 *   LDcsc2csrMySpMatrix(Double)    src/formatConvert.cpp:300-398 (assumes
 *                                  nzmax == nnz, narrows to float / keeps double)
 *   LDcsc2cscMySpMatrix            src/formatConvert.cpp:334-365
 *
 * Outputs are malloc'd, as the reference's (released with mySpMatrixFree or
 * free by the caller).
 */
#ifndef GG_COMPAT_FORMAT_CONVERT_H_
#define GG_COMPAT_FORMAT_CONVERT_H_

#include "SpMV.h"

class ucr_cs_dl {
public:
    long int nzmax;   /* maximum number of entries */
    long int m;       /* number of rows */
    long int n;       /* number of columns */
    long int *p;      /* column pointers (size n+1) */
    long int *i;      /* row indices, size nzmax */
    double *x;        /* numerical values, size nzmax */
    long int nz;
    void shallowCpy(long int nzmaxIn, long int mIn, long int nIn, long int *pIn, long int *iIn,
                    double *xIn, long int nzIn)
    {
        nzmax = nzmaxIn;
        m = mIn;
        n = nIn;
        p = pIn;
        i = iIn;
        x = xIn;
        nz = nzIn;
    }
};

void coo2csr_in(int numRows, int nz, float *a, int *i_idx, int *j_idx);
void coo2csrDouble_in(int numRows, int nz, double *a, int *i_idx, int *j_idx);
void LDcsc2csrMySpMatrix(MySpMatrix *mySpM, ucr_cs_dl *M);
void LDcsc2cscMySpMatrix(MySpMatrix *mySpM, ucr_cs_dl *M);
void LDcsc2csrMySpMatrixDouble(MySpMatrixDouble *mySpM, ucr_cs_dl *M);

#endif /* GG_COMPAT_FORMAT_CONVERT_H_ */
