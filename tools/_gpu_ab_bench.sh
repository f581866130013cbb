# A/B of bench variants (env settings) in one call
set -e
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > gpurun_out/ab/b$i.json 2> gpurun_out/ab/b$i.err
  echo "$v: $(python3 -c "import json;d=json.load(open('gpurun_out/ab/b$i.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"
done
