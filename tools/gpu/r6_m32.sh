# 32-row ws tiles: conv tests, then per-shape bench (TLOD_BENCH_SHAPES=1) and bench A/B vs
# the m32off variant.  usage: bash tools/gpu/r6_m32.sh OUTDIR
set -e
O=${1:-gpurun_out/r6m32}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_conv_bs_gpu.py tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/shapes_new.json 2> $O/shapes_new.err
TLOD_LIB=build_variants/m32off/libtlod.so TLOD_BENCH_SHAPES=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/shapes_old.json 2> $O/shapes_old.err
grep -E "fwd|dgrad" $O/shapes_new.err | sort > $O/sn.txt; grep -E "fwd|dgrad" $O/shapes_old.err | sort > $O/so.txt
paste -d'|' $O/sn.txt $O/so.txt | awk -F'|' '{print $1 "   <- new | old ->  " $2}' | grep "bf16x6   \|dgrad/bf16x6" | head -30
bash tools/gpu/r6_ab.sh $O/ab 2 m32off "daf vgg16" "daf res101"
