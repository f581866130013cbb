set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for res in 0 32; do
  TLOD_CU_RESERVE=$res timeout -k 10 300 python3 tools/overlap_probe.py --steps 5 --contend --contend-wgs 32 > $O/contend_r$res.json 2> $O/contend_r$res.err
  python3 -c "import json;d=json.load(open('$O/contend_r$res.json'));print('reserve', $res, d['contention'])"
done
for res in 0 16 32; do
  TLOD_CU_RESERVE=$res timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/bench_r$res.json 2>/dev/null
  python3 -c "import json;d=json.load(open('$O/bench_r$res.json'));print('reserve', $res, 'bench', d['value'])"
done
