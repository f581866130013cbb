# final refresh: configs 3-5 lines and the R101 kernel stats on the final tree
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "daf res101" "maf vgg16" "atf res101"; do
  set -- $cfg
  timeout -k 10 400 python3 bench.py --method $1 --net $2 --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err
  python3 -c "import json;d=json.loads(open('$O/bench_$1_$2.json').read().strip().splitlines()[-1]);print('$1 $2', d['value'])"
done
bash tools/gpu/profile_r101.sh $O/r101 > $O/r101_busy.txt 2>&1 || true
tail -4 $O/r101_busy.txt
