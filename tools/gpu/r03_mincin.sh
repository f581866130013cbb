# Round-3 lease: warp-specialized conv for Cin = 64 (TLOD_WS_MINCIN=64: conv1_2 / conv2_1)
# and frame-aligned split-K pieces — conv tests, microbench, bench A/B.
# usage: bash tools/gpu/r03_mincin.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_conv_bs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2; do
  for v in 128 64; do
    for shp in "--C 64 --H 300 --W 600" "--C 512 --H 37 --W 75"; do
      echo "mincin=$v $shp $(TLOD_WS_MINCIN=$v timeout -k 10 120 python tools/bench_conv.py --math bf16x6 $shp 2>/dev/null)"
    done
  done
done > $O/micro.txt 2>&1
cat $O/micro.txt | cut -c1-160
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "m128=." "m64=.:TLOD_WS_MINCIN=64" > $O/ab.txt 2>&1
cat $O/ab.txt
