# Round-3 lease: ResNet101 ReLU backward folded into the 3x3 conv2 dgrad (TLOD_FUSE_RELU=0/1):
# R101 / ATF / MAF step tests, DAF-R101 bench A/B.  usage: bash tools/gpu/r03_r101fuse.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py tests/test_atf_step_gpu.py tests/test_conv_bs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2 3; do
  for f in 0 1; do
    TLOD_FUSE_RELU=$f timeout -k 10 400 python3 bench.py --net res101 --steps 8 --warmup 2 --cpu-baseline-steps 0 > $O/b_${f}_${r}.json 2> $O/b_${f}_${r}.err
    echo "fuse=$f r$r: $(python3 -c "import json;d=json.load(open('$O/b_${f}_${r}.json'));print(d['value'], d['ms_per_step'], d['fused_relu_backward_per_step'])")"
  done
done
