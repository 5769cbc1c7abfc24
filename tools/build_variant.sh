#!/bin/bash
# build the library from another source directory into lib/exp/NAME.so (A/B experiments; run
# on the CPU side, the .so travels with the snapshot).  usage: tools/build_variant.sh NAME SRC_DIR [FLAGS...]
set -e
NAME=$1; SRC=$2; shift 2
PKG=/root/repo/julia-ocean-modelling_amd
OUT=/tmp/variant_$NAME; rm -rf $OUT; mkdir -p $OUT $PKG/lib/exp
for f in qg_stencil qg_spectral qg_pcg qg_capi qg_comm qg_diag qg_mg; do
  X=""; [ $f = qg_stencil ] && X="-ffp-contract=off"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I/root/repo/include -I$SRC -Wall -Wno-unused-function $X "$@" -c $SRC/$f.hip -o $OUT/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $PKG/lib/exp/$NAME.so $OUT/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
ls -la $PKG/lib/exp/$NAME.so
