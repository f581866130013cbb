# RoIAlignAvg backward: the RoI GPU tests, then the microbench new vs old (variant) build,
# and the kernel stats of the new one.
set -e
O=${1:-gpurun_out/r6r}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 60 python3 tools/bench_roi.py
  TLOD_LIB=build_variants/head/libtlod.so timeout -k 10 60 python3 tools/bench_roi.py
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 tools/bench_roi.py > /dev/null 2>&1
python3 -c "
import csv
for r in csv.DictReader(open('$O/stats/run_kernel_stats.csv')):
    print('%8.1f us %5s calls  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))
"
