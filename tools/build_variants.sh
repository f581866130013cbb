#!/bin/bash
# Build libtlod.so variants with extra -D flags for A/B timing (load with TLOD_LIB=path).
# usage: tools/build_variants.sh NAME "-DFOO=1 -DBAR=2"
#        CONV_SRC=/path/conv.hip tools/build_variants.sh NAME   (another conv.hip, e.g. HEAD's)
set -e
cd "$(dirname "$0")/../transfer-learning-library-for-object-detection_amd/csrc"
make -j8 >/dev/null
name=$1; shift
out=../../build_variants/$name
mkdir -p $out
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I. $*"
/opt/rocm/bin/hipcc $FLAGS -c ${CONV_SRC:-conv.hip} -o $out/conv.o
/opt/rocm/bin/hipcc $FLAGS -c gemm.hip -o $out/gemm.o
objs=$(ls build/*.o | grep -v '/conv.o$' | grep -v '/gemm.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libtlod.so $out/conv.o $out/gemm.o $objs
echo $out/libtlod.so
