#!/bin/bash
# Build an alternative libfrm for an A/B into fractal-ray-marching_amd/ab/NAME.so without touching
# lib/libfrm.so: extra compile flags and/or a patch applied to a copy of csrc/ (experiments live as
# patches under profiles/, never in the product sources). Delete ab/ after the A/B: every gpurun
# call ships it.
# Usage: PATCH=profiles/round4/ab_prio/prio.patch bash tools/build_variant.sh NAME "-DFOO=1 ..."
# (SCHEDFLAGS=... in the environment replaces the Makefile's scheduler options, e.g. SCHEDFLAGS="")
# (MAKEVARS="RING_WAVES=8 ..." passes Makefile variables)
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/fractal-ray-marching_amd"
SRC=csrc
if [ -n "$PATCH" ]; then
  SRC=build/src_$NAME
  rm -rf "$SRC"; mkdir -p "$SRC"
  cp csrc/* "$SRC/"
  (cd "$SRC" && patch -s -p3 < "$ROOT/$PATCH")
fi
OBJ=build/obj_$NAME
mkdir -p ab
make -s CSRC="$SRC" OBJDIR=$OBJ EXTRA_HIPFLAGS="$FLAGS" $MAKEVARS ${SCHEDFLAGS+SCHEDFLAGS="$SCHEDFLAGS"} $OBJ/frm_kernels.o $OBJ/frm_api.o \
  $OBJ/frm_sched.o $OBJ/frm_host.o $OBJ/frm_reload.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ab/$NAME.so $OBJ/frm_kernels.o \
  $OBJ/frm_api.o $OBJ/frm_sched.o $OBJ/frm_host.o $OBJ/frm_reload.o -lhiprtc -lrccl
echo "ab/$NAME.so"
