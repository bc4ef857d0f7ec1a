#!/bin/bash
# tools/build_variant.sh NAME -DMACRO=V ...  -> variants/libggmres_NAME.so
# (kernels.hip rebuilt with the given macros, other objects from the main build;
# select at run time with GGMRES_LIB=variants/libggmres_NAME.so; VARDIR=abvar puts
# it in abvar/ instead, which travels to the GPU box -- variants/ does not)
set -e
cd "$(dirname "$0")/../gpu-gmres_amd"
name=$1; shift
VD=${VARDIR:-variants}
mkdir -p ../$VD build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -I../include/compat -I../include -Icsrc \
    "$@" -c csrc/kernels.hip -o build/var/kernels_$name.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../$VD/libggmres_$name.so build/var/kernels_$name.o \
    $(find build -name "*.o" ! -path "build/var/*" ! -name kernels.o | sort) -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
