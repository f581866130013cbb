# Round-3 lease: RoIAlignAvg gather backward, 1x1 tile choice, 16x16x16 GEMM variant — op /
# conv / ResNet / linear tests, bench A/B (gather vs atomic; GEMM 32x32 vs 16x16), DAF-R101
# line, RoI backward microbench.  usage: bash tools/gpu/r03_roi.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_conv_bs_gpu.py tests/test_resnet_gpu.py tests/test_linear_gpu.py tests/test_rpn_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
TLOD_LIB=build_variants/mf16/libtlod.so timeout -k 10 300 python -u -m pytest tests/test_linear_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_mf16.log 2>&1
tail -2 $O/pytest_mf16.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 2 "atomic=." "gather=.:TLOD_ROI_BWD_GATHER=1" > $O/ab.txt 2>&1
cat $O/ab.txt
TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --net res101 --cpu-baseline-steps 0 > $O/r101.json 2> $O/r101.err
echo "r101: $(python3 -c "import json;d=json.load(open('$O/r101.json'));print(d['value'], d['ms_per_step'])")"
timeout -k 10 120 python3 tools/bench_roi.py > $O/roi.txt 2> $O/roi.err
TLOD_ROI_BWD_GATHER=1 timeout -k 10 120 python3 tools/bench_roi.py >> $O/roi.txt 2>> $O/roi.err
cat $O/roi.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/roistats -o run -- python3 tools/bench_roi.py > /dev/null 2> $O/roistats.err
