# Interleaved A/B of bench.py configs between this tree and a variant library.
# usage: bash tools/gpu/r6_ab.sh OUTDIR ROUNDS VARIANT "method net" ...
set -e
O=$1; R=$2; V=$3; shift 3
CFGS=("$@")
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    for lab in new $V; do
      labf=${lab//[:=]/_}
      if [ $lab = new ]; then L=""; elif [ "${V#env:}" != "$V" ]; then L="${V#env:}"; else L="TLOD_LIB=build_variants/$V/libtlod.so"; fi
      env $L timeout -k 10 300 python3 bench.py --method $1 --net $2 --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/$1_$2_$labf.$r.json 2> $O/$1_$2_$labf.$r.err
      echo "$1 $2 $lab r$r: $(python3 -c "import json;d=json.load(open('$O/$1_$2_$labf.$r.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
