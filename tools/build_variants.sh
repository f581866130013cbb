#!/bin/bash
# Build libtlod.so variants with extra -D flags for A/B timing (load with TLOD_LIB=path).
# usage: tools/build_variants.sh NAME "-DFOO=1 -DBAR=2"
#        CONV_SRC=/path/conv.hip tools/build_variants.sh NAME   (another conv.hip, e.g. HEAD's)
#        EXTRA_SRCS="optim.hip" tools/build_variants.sh NAME -DTLOD_SGD_NT=0
set -e
cd "$(dirname "$0")/../transfer-learning-library-for-object-detection_amd/csrc"
make -j8 >/dev/null
name=$1; shift
out=../../build_variants/$name
mkdir -p $out
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I. $*"
/opt/rocm/bin/hipcc $FLAGS -c ${CONV_SRC:-conv.hip} -o $out/conv.o
/opt/rocm/bin/hipcc $FLAGS -c gemm.hip -o $out/gemm.o
# EXTRA_SRCS="optim.hip act.hip": more sources rebuilt with the flags
extra=""
excl="-e /conv.o$ -e /gemm.o$"
for src in ${EXTRA_SRCS:-}; do
  b=$(basename $src .hip)
  /opt/rocm/bin/hipcc $FLAGS -c $src -o $out/$b.o
  extra="$extra $out/$b.o"
  excl="$excl -e /$b.o$"
done
objs=$(ls build/*.o | grep -v $excl)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libtlod.so $out/conv.o $out/gemm.o $extra $objs
echo $out/libtlod.so
