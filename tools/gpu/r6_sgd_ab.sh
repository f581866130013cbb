# Optimizer microbench + DAF-VGG16 A/B of this tree vs a variant library.
# usage: bash tools/gpu/r6_sgd_ab.sh OUTDIR VARIANT ROUNDS
set -e
O=$1; V=$2; R=$3
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for lab in new $V; do
    if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$V/libtlod.so"; fi
    env $L timeout -k 10 120 python3 tools/bench_sgd.py > $O/sgd_$lab.$r.json 2> $O/sgd_$lab.$r.err
    echo "sgd $lab r$r: $(cat $O/sgd_$lab.$r.json)"
  done
done
bash tools/gpu/r6_ab.sh $O/ab $R $V "daf vgg16"
