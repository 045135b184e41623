#!/bin/bash
# build_variant.sh NAME [extra hipcc flags...] -> build_variants/NAME/libmvc_hip.so
# (tuning aid: run the bench against it with MVC_HIP_LIB=...)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/build_variants/$NAME; mkdir -p $OUT
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I$ROOT/include -I$ROOT/multiview-clustering_amd/csrc -w $*"
S=$ROOT/multiview-clustering_amd/csrc
for f in mvc_exact mvc_parallel mvc_spec mvc_ari mvc_synth; do /opt/rocm/bin/hipcc $F -c $S/$f.hip -o $OUT/$f.o & done
/opt/rocm/bin/hipcc $F -x hip -c $S/mvc_api.cpp -o $OUT/mvc_api.o &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/libmvc_hip.so $OUT/mvc_exact.o $OUT/mvc_parallel.o $OUT/mvc_spec.o $OUT/mvc_ari.o $OUT/mvc_synth.o $OUT/mvc_api.o
rm -f $OUT/*.o
