# GEMM second-half interleave (sched_group_barrier: MFMA, N VALU, 1 LDS store) variants vs
# the pinned-block default (new) and HEAD (ghead)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in new sgb6; do
  L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
  TLOD_LIB=$L timeout -k 10 600 python3 -u -m pytest tests/test_linear_gpu.py tests/test_conv_bs_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.$v.log 2>&1 || { tail -30 $O/pytest.$v.log; exit 1; }
  tail -1 $O/pytest.$v.log
done
for r in 1 2; do
  for v in new ghead sgb4 sgb6 sgb10; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    echo "$v fc   $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py 2>/dev/null)"
    echo "$v r101 $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py --r101 2>/dev/null)"
    echo "$v x $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_1x1.py 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.load(sys.stdin)["total_ms"])')"
  done
done
