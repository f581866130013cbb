# Round-3 lease: 1x1 split-bf16 conv GEMM — conv / ResNet tests, bench A/B (TLOD_CONV1X1_BS)
# on DAF-VGG16 and DAF-ResNet101.  usage: bash tools/gpu/r03_1x1.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_conv_bs_gpu.py tests/test_conv_gpu.py tests/test_resnet_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 600 bash tools/gpu/ab.sh $O/ab 2 "on=." "off=.:TLOD_CONV1X1_BS=0" > $O/ab.txt 2>&1
cat $O/ab.txt
for arm in on off; do
  env=""; [ $arm = off ] && env="TLOD_CONV1X1_BS=0"
  env $env TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --net res101 --cpu-baseline-steps 0 > $O/r101_$arm.json 2> $O/r101_$arm.err
  echo "r101 $arm: $(python3 -c "import json;d=json.load(open('$O/r101_$arm.json'));print(d['value'], d['ms_per_step'])")"
done
