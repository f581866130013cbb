# Round-3 lease: RoIAlignAvg backward — the tap-segment gather (default) vs the atomic
# kernels: op tests, DAF step tests, microbench, bench A/B.  usage: bash tools/gpu/r03_roi.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_daf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2; do
  TLOD_ROI_BWD_GATHER=0 timeout -k 10 60 python3 tools/bench_roi.py
  timeout -k 10 60 python3 tools/bench_roi.py
done
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "atomic=.:TLOD_ROI_BWD_GATHER=0" "gather=." > $O/ab.txt 2>&1
cat $O/ab.txt
