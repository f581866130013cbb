# conv1_1 direct kernel A/B: tools/bench_direct.py per variant, then DAF-VGG16 vs the best.
# usage: bash tools/gpu/r6_direct_ab.sh OUTDIR ROUNDS VARIANT...
set -e
O=$1; R=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for lab in new "$@"; do
    if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
    echo "$lab r$r: $(env $L timeout -k 10 120 python3 tools/bench_direct.py 2> $O/d_$lab.$r.err)"
  done
done
