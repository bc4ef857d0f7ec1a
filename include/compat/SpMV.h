/*
 * compat/SpMV.h -- the two sparse-matrix holder classes the reference's PG
 * boundary passes around, with the reference's exact member layout
 * (src/SpMV.h:57-102, include guard included).  A caller that already has the
 * reference's SpMV.h on its include path uses that one instead; both define
 * the same layout (checked by static_assert in compat/interface_pg.cpp).
 */
#ifndef __SPMV_H__
#define __SPMV_H__

/* src/SpMV.h:22-54: the triplet holder and the device CSR the engine ABI
 * (GMRES_GPU(SpMatrixGPU*, SpMatrix*, ...), compat/gmres.h) receives */
struct nzInfo {
    int rowNum;
    int colNum;
    float val;
};
typedef struct nzInfo NZEntry;

struct SpM {
    int numRows;
    int numCols;
    int numNZEntries;
    NZEntry *nzentries;
    int *rowPtrs;
    int *colPtrs;
};
typedef struct SpM SpMatrix;

struct SpMGPU {
    float *d_val;
    int *d_indices;
    int *d_rowIndices;
    int *d_ins_indices;
    int *d_ins_rowIndices;
    int *d_ins_inputList;
};
typedef struct SpMGPU SpMatrixGPU;

class MySpMatrix {
public:
    int isCSR;
    int numRows;
    int numCols;
    int numNZEntries;
    float *d_val;
    int *d_indices;
    int *d_rowIndices;
    float *val;
    int *indices;
    int *rowIndices;
    void Initilize(SpMatrix &M);   /* defined by the caller's mySpMatrix.cu */
};

class MySpMatrixDouble {
public:
    int isCSR;
    int numRows;
    int numCols;
    int numNZEntries;
    double *d_val;
    int *d_indices;
    int *d_rowIndices;
    double *val;
    int *indices;
    int *rowIndices;
};

#endif /* __SPMV_H__ */
