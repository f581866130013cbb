# Round 6: run selected GPU test files, then the conv3_3 microbench.
# usage: bash tools/gpu/r6_tests.sh OUTDIR "test files..."
set -e
O=${1:-gpurun_out/r6t}; shift
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest $@ -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python3 tools/bench_conv.py --math bf16x6 > $O/conv33.json 2> $O/conv33.err
cat $O/conv33.json
