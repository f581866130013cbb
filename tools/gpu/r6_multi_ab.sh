# Interleaved A/B of several variant libraries: conv3_3 microbench + DAF-VGG16 step.
# usage: bash tools/gpu/r6_multi_ab.sh OUTDIR ROUNDS VARIANT...
set -e
O=$1; R=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for lab in new "$@"; do
    if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
    env $L timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 > $O/c_$lab.$r.json 2>/dev/null
    env $L timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/b_$lab.$r.json 2>/dev/null
    echo "$lab r$r: $(python3 -c "import json;d=json.load(open('$O/b_$lab.$r.json'));c=json.load(open('$O/c_$lab.$r.json'));print(d['value'], c['dgrad_ms'], c['wgrad_ms'], c['fwd_ms'])")"
  done
done
