# conv1_1 direct conv: nontemporal output stores (new) vs plain (directold)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_conv_bs_gpu.py -x -q -k "direct" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new directold; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 > $O/daf.$v.$r.json 2>/dev/null
    echo "$v r$r daf $(python3 -c "import json;print(json.load(open('$O/daf.$v.$r.json'))['value'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new directold; do
  L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
  TLOD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline-steps 0 > /dev/null 2>&1
  python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
    if 'direct' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000,1))
"
done
