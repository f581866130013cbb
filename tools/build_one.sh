#!/bin/bash
# Variant of libtlod.so with ONE source rebuilt under extra -D flags (faster than
# build_variants.sh, which rebuilds conv.hip and gemm.hip too).
# usage: tools/build_one.sh NAME SRC.hip "-DFOO=1 ..."   -> build_variants/NAME/libtlod.so
set -e
cd "$(dirname "$0")/../transfer-learning-library-for-object-detection_amd/csrc"
make -j8 >/dev/null
name=$1; src=$2; shift 2
out=../../build_variants/$name
mkdir -p $out
b=$(basename $src .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I. "$@" -c $src -o $out/$b.o
objs=$(ls build/*.o | grep -v "/$b.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libtlod.so $out/$b.o $objs
echo $out/libtlod.so
