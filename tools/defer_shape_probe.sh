#!/bin/bash
# Builds variants of libsimilarity_transform.so with other deferred-round
# launch shapes (st_kernels.hip ST_DEFER_* macros) into eigen_value_amd/lib/variants/NAME,
# for timing the real solve loop with EIGEN_VALUE_LIB=... (tools/defer_profile.py).
#   bash tools/defer_shape_probe.sh NAME "-DST_DEFER_R0_CACHED=4 ..."
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/build/variants/$NAME; OUT=$ROOT/eigen_value_amd/lib/variants/$NAME; mkdir -p $OBJ $OUT
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$ROOT/include -I$ROOT/eigen_value_amd/csrc"
for f in st_kernels st_solve st_multi; do
  /opt/rocm/bin/hipcc $FL -DST_PROBES=1 $DEFS -c $ROOT/eigen_value_amd/csrc/$f.hip -o $OBJ/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libsimilarity_transform.so $OBJ/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libsimilarity_transform.so"
