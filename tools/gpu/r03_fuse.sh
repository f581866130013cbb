# Round-3 lease: fused ReLU-backward dgrad + wgrad bias gradient, RoI gather v2, at_sample digit
# search — tests, then bench A/B against round-2 HEAD and the gather knob, RoI microbench.
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_conv_bs_gpu.py tests/test_conv_gpu.py tests/test_ops_gpu.py tests/test_rpn_gpu.py tests/test_daf_step_gpu.py tests/test_frcnn_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 2 "head=build_variants/head" "new=." "gather=.:TLOD_ROI_BWD_GATHER=1" > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 120 python3 tools/bench_roi.py > $O/roi.txt 2> $O/roi.err
TLOD_ROI_BWD_GATHER=1 timeout -k 10 120 python3 tools/bench_roi.py >> $O/roi.txt 2>> $O/roi.err
cat $O/roi.txt
