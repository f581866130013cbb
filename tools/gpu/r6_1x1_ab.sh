# 1x1 conv planner A/B: tools/bench_1x1.py and DAF-R101 bench per variant library.
# usage: bash tools/gpu/r6_1x1_ab.sh OUTDIR ROUNDS VARIANT...
set -e
O=$1; R=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for lab in new "$@"; do
    if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
    env $L timeout -k 10 120 python3 tools/bench_1x1.py > $O/b1x1_$lab.$r.json 2> $O/b1x1_$lab.$r.err
    env $L timeout -k 10 300 python3 bench.py --method daf --net res101 --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/daf_r101_$lab.$r.json 2> $O/daf_r101_$lab.$r.err
    echo "$lab r$r: $(python3 -c "import json;d=json.load(open('$O/daf_r101_$lab.$r.json'));b=json.load(open('$O/b1x1_$lab.$r.json'));print(d['value'], b['total_ms'])")"
  done
done
