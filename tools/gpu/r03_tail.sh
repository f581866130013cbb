# Round-3 lease: vectorized tail reduces — conv / linear tests, bench A/B vs the previous
# commit (build_variants/prev).  usage: bash tools/gpu/r03_tail.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_conv_bs_gpu.py tests/test_conv_gpu.py tests/test_linear_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "prev=build_variants/prev" "new=." > $O/ab.txt 2>&1
cat $O/ab.txt
