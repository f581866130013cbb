# Round-3 lease: how much of the warp-specialized conv is its epilogue store (timing-only
# no-store build) and how the 150 x 250 tile choice compares with 16 x 32 tiles.
# usage: bash tools/gpu/r03_epi.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in base nostore flex0; do
    envs=""; [ $v = nostore ] && envs="TLOD_LIB=build_variants/nostore/libtlod.so"
    [ $v = flex0 ] && envs="TLOD_WS_FLEX=0"
    for shp in "--C 256 --H 150 --W 250" "--C 256 --H 150 --W 300" "--C 512 --H 75 --W 150"; do
      echo "$v $shp $(env $envs timeout -k 10 120 python tools/bench_conv.py --math bf16x6 $shp 2>/dev/null)"
    done
  done
done > $O/micro.txt 2>&1
cat $O/micro.txt
