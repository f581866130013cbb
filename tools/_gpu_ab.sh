set -e
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in "" "build_variants/nomid/libtlod.so"; do
  echo "== variant ${v:-default}"
  TLOD_LIB=$v timeout -k 10 120 python -u tools/bench_conv.py --math bf16x6
  TLOD_LIB=$v timeout -k 10 120 python -u tools/bench_conv.py --math bf16x6 --C 512 --H 37 --W 75
  TLOD_LIB=$v timeout -k 10 120 python -u tools/bench_gemm.py
done > gpurun_out/ab.log 2>&1
