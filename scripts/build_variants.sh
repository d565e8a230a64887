#!/bin/bash
# Build libtde variants that differ only in conv_igemm.hip compile-time knobs (diagnostic A/B).
#   bash scripts/build_variants.sh NAME "-DFLAG=V ..." [NAME "-D..." ...]  -> variants/libtde_NAME.so
set -eu
cd "$(dirname "$0")/../tf_depth_estimation_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../variants
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $FLAGS -c conv_igemm.hip -o build/conv_$NAME.o
  OBJS=$(ls build/*.o | grep -v "build/conv_" | grep -v conv_igemm.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../variants/libtde_$NAME.so build/conv_$NAME.o $OBJS
  echo "built variants/libtde_$NAME.so ($FLAGS)"
done
