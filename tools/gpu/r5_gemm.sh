# Round 5: GEMM K-image swizzle + fused residual epilogue — tests, bench_gemm A/B vs
# build_variants/base, PMC; then the conv3_3 dgrad / wgrad stream pair.
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests/test_linear_gpu.py tests/test_conv_bs_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_gemm.py > $O/gnew.$r.json; echo "new  $(cat $O/gnew.$r.json)"
  TLOD_LIB=build_variants/base/libtlod.so timeout -k 10 120 python3 tools/bench_gemm.py > $O/gbase.$r.json; echo "base $(cat $O/gbase.$r.json)"
done
timeout -k 10 120 python3 tools/bench_gemm.py --r101 > $O/gnew_r101.json; echo "new r101 $(cat $O/gnew_r101.json)"
TLOD_LIB=build_variants/base/libtlod.so timeout -k 10 120 python3 tools/bench_gemm.py --r101 > $O/gbase_r101.json; echo "base r101 $(cat $O/gbase_r101.json)"
bash tools/gpu/pmc_gemm.sh $O/pmc > /dev/null
cat $O/pmc/p2.txt | head -8
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/pair.$r.json; cat $O/pair.$r.json
  TLOD_CONV_KSPLIT_MAX=1 timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/nosplit.$r.json; cat $O/nosplit.$r.json
done
