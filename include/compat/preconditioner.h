/*
 * compat/preconditioner.h -- the reference's preconditioner plug-in base class
 * (src/preconditioner.h:34-84, include guard included) with its exact layout:
 * vtable pointer, numRows, then the GMRES workspace pointers, and the virtual
 * functions in declaration order (the vtable is ABI).  A caller derives its
 * preconditioner from this class and passes it to the engines of
 * compat/gmres.h, which call its Dev* / Host* methods.
 *
 * The reference's own subclasses (MyAINV / MyILU0 / MyILUK over cusp and the
 * legacy cuSPARSE, MyILUPP / MyILUPPfloat over ILU++) are not provided: the
 * library's built-in preconditioners are gg_set_precond_* (ggmres.h) and the PG
 * classes (gmres_interface_pg.h).  Note: the thermal testbed's src_thermal/
 * carries a DIFFERENT class of the same name (three virtuals, no workspace
 * pointers, src_thermal/preconditioner.h:36-66); this header is src/'s.
 */
#ifndef PRECONDITIONER_H_
#define PRECONDITIONER_H_

#include "SpMV.h"

class Preconditioner {
public:
    typedef int IndexType;
    typedef float ValueType;

    int numRows;

    /* ---- For GMRES --- (workspace the reference's engines borrow,
       src/gmres.cu:2285-2286,2337-2339; libggmres's engines keep their own) */
    float *d_r, *d_rr, *d_bb, *d_y;
    float *s, *cs, *sn, *H;
    float *d_v, *d_w, *d_ww;

    virtual void HostPrecond(const ValueType *i_data, ValueType *o_data) = 0;
    virtual void DevPrecond(const ValueType *i_data, ValueType *o_data) = 0;
    virtual void Initilize(const MySpMatrix &mySpM) = 0;

    virtual void HostPrecond_rhs(const ValueType *i_data, ValueType *o_data) = 0;
    virtual void HostPrecond_right(const ValueType *i_data, ValueType *o_data) = 0;
    virtual void HostPrecond_left(const ValueType *i_data, ValueType *o_data) = 0;
    virtual void HostPrecond_starting_value(const ValueType *i_data, ValueType *o_data) = 0;

    virtual void DevPrecond_rhs(float *i_data, float *o_data) = 0;
    virtual void DevPrecond_right(float *i_data, float *o_data) = 0;
    virtual void DevPrecond_left(float *i_data, float *o_data) = 0;
    virtual void DevPrecond_starting_value(float *i_data, float *o_data) = 0;

    virtual ~Preconditioner() {}
};

#endif /* PRECONDITIONER_H_ */
