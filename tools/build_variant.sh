#!/bin/bash
# Build an alternative libfrm (extra compile flags) into fractal-ray-marching_amd/variants/NAME.so
# without touching lib/libfrm.so. Usage: bash tools/build_variant.sh NAME "-DFOO=1 ..."
# (SCHEDFLAGS=... in the environment replaces the Makefile's scheduler options, e.g. SCHEDFLAGS="")
set -e
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../fractal-ray-marching_amd"
mkdir -p variants
make -s OBJDIR=build/obj_$NAME EXTRA_HIPFLAGS="$FLAGS" ${SCHEDFLAGS+SCHEDFLAGS="$SCHEDFLAGS"} build/obj_$NAME/frm_kernels.o build/obj_$NAME/frm_api.o \
  build/obj_$NAME/frm_sched.o build/obj_$NAME/frm_host.o build/obj_$NAME/frm_reload.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/$NAME.so build/obj_$NAME/frm_kernels.o \
  build/obj_$NAME/frm_api.o build/obj_$NAME/frm_sched.o build/obj_$NAME/frm_host.o build/obj_$NAME/frm_reload.o -lhiprtc
echo "variants/$NAME.so"
