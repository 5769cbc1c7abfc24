#!/bin/bash
# build an experiment variant of the library: buildexp.sh NAME FLAGS...
cd /root/repo/julia-ocean-modelling_amd
NAME=$1; shift
OUT=exp/$NAME; mkdir -p $OUT
for f in qg_stencil qg_spectral qg_pcg qg_capi qg_comm qg_diag; do
  X=""; [ $f = qg_stencil ] && X="-ffp-contract=off"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I../include -I${CSRC:-csrc} -Wall -Wno-unused-function $X "$@" -c ${CSRC:-csrc}/$f.hip -o $OUT/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libqgmi355.so $OUT/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
ls -la $OUT/libqgmi355.so
