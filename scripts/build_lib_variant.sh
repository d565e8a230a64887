#!/bin/bash
# Whole-library build variant (all translation units with extra compile flags) for A/B runs:
#   bash scripts/build_lib_variant.sh NAME "-DFLAG=V ..."   -> variants/libtde_NAME.so  (load with TDE_LIBRARY=...)
set -eu
cd "$(dirname "$0")/../tf_depth_estimation_amd/csrc"
NAME=$1; FLAGS=$2
B=build_$NAME
mkdir -p $B ../../variants
ls *.hip | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $FLAGS -c {} -o $B/\$(basename {} .hip).o"
g++ -O3 -std=c++17 -fPIC -Wall -c host_util.cpp -o $B/host_util.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../variants/libtde_$NAME.so $B/*.o
rm -rf $B
echo "built variants/libtde_$NAME.so ($FLAGS)"
