# Interleaved A/B of several variant libraries on given bench configs.
# usage: bash tools/gpu/r6_cfg_ab.sh OUTDIR ROUNDS "VARIANTS" "method net" ...
set -e
O=$1; R=$2; VS=$3; shift 3
CFGS=("$@")
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    for lab in new $VS; do
      if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
      env $L timeout -k 10 300 python3 bench.py --method $1 --net $2 --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/$1_$2_$lab.$r.json 2>/dev/null
      echo "$1 $2 $lab r$r: $(python3 -c "import json;d=json.load(open('$O/$1_$2_$lab.$r.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
