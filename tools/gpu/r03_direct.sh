# Round-3 lease: direct conv1_1 kernel + knob A/Bs (fused ReLU backward, RoI gather) with
# per-shape conv timings.  usage: bash tools/gpu/r03_direct.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_bs_gpu.py -x -q --timeout 300 --timeout-method thread -k "direct or fused or masked" > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "new=." "nofuse=.:TLOD_FUSE_RELU=0" > $O/ab.txt 2>&1
cat $O/ab.txt
TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/shapes_new.json 2> $O/shapes_new.err
TLOD_FUSE_RELU=0 TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/shapes_nofuse.json 2> $O/shapes_nofuse.err
echo shapes done
