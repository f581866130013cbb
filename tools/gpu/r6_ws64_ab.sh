# ws kernel for Cin = 64 (-DTLOD_WS_MINCIN=64): conv tests under the variant, per-shape conv
# times (TLOD_BENCH_SHAPES=1) and the step A/B.  usage: bash tools/gpu/r6_ws64_ab.sh OUTDIR ROUNDS
set -e
O=$1; R=$2
mkdir -p $O
export PYTHONUNBUFFERED=1
V=ws64
TLOD_LIB=build_variants/$V/libtlod.so timeout -k 10 400 python3 -m pytest tests/test_conv_bs_gpu.py -q -x --timeout 200 --timeout-method thread > $O/t_$V.log 2>&1 || { tail -20 $O/t_$V.log; exit 1; }
echo "tests $V: $(tail -1 $O/t_$V.log)"
for lab in new $V; do
  if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
  env $L TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/shapes_$lab.json 2> $O/shapes_$lab.err
  grep "64, 600, 1200\|64, 300, 600" $O/shapes_$lab.err | sed "s/^/$lab /"
done
bash tools/gpu/r6_ab.sh $O/ab $R $V "daf vgg16" "daf res101"
