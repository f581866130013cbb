# Interleaved A/B of bench.py between trees / env settings in one lease.
# usage: bash tools/gpu/ab.sh OUTDIR ROUNDS "label=dir[:ENV=V ...]" ...
set -e
O=$1; R=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 $R); do
  for spec in "$@"; do
    lab=${spec%%=*}; rest=${spec#*=}; dir=${rest%%:*}; envs=""
    [ "$rest" != "$dir" ] && envs=${rest#*:}
    ( cd "$dir" && env $envs timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 ) > $O/$lab.$r.json 2> $O/$lab.$r.err
    echo "$lab r$r: $(python3 -c "import json;d=json.load(open('$O/$lab.$r.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"
  done
done
