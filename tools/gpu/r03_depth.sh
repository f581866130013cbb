# Round-3 lease: producer prefetch depth 2 vs 1 (build_variants/depth1)
# bench A/B.  usage: bash tools/gpu/r03_frame.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_conv_bs_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2; do
  for v in depth1 depth2; do
    envs=""; [ $v = depth1 ] && envs="TLOD_LIB=build_variants/depth1/libtlod.so"
    for shp in "--C 256 --H 150 --W 250" "--C 256 --H 150 --W 300" "--C 512 --H 75 --W 150" "--C 512 --H 37 --W 75"; do
      echo "$v $shp $(env $envs timeout -k 10 120 python tools/bench_conv.py --math bf16x6 $shp 2>/dev/null)"
    done
  done
done > $O/micro.txt 2>&1
cat $O/micro.txt | cut -c1-160
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "depth1=.:TLOD_LIB=build_variants/depth1/libtlod.so" "depth2=." > $O/ab.txt 2>&1
cat $O/ab.txt
