#!/bin/bash
# Variant of libtlod.so with several sources rebuilt under extra -D flags.
# usage: tools/build_multi.sh NAME "-DFOO=1 ..." SRC1.hip [SRC2.hip ...] -> build_variants/NAME/libtlod.so
set -e
cd "$(dirname "$0")/../transfer-learning-library-for-object-detection_amd/csrc"
make -j8 >/dev/null
name=$1; flags=$2; shift 2
out=../../build_variants/$name
mkdir -p $out
excl=""
for src in "$@"; do
  b=$(basename $src .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I. $flags -c $src -o $out/$b.o &
  excl="$excl|/$b.o$"
done
wait
objs=$(ls build/*.o | grep -Ev "${excl#|}")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libtlod.so $out/*.o $objs
rm -f $out/*.o
echo $out/libtlod.so
