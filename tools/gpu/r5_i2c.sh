# im2col / col2im with 32-bit index arithmetic (new) vs 64-bit (rshead)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_resnet_gpu.py -x -q -k "im2col or head" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new rshead; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.$r.json 2>/dev/null
    echo "$v r$r atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.$r.json'))['value'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --method atf --net res101 --steps 3 --warmup 1 --cpu-baseline-steps 0 > /dev/null 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'im2col' in r['Name'] or 'col2im' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1000,1))
"
