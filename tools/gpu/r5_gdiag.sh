# GEMM timing-only ablations: 1 = no global loads in the K loop, 2 = no split (raw bits), 3 = no LDS staging stores
set -e
O=$1; mkdir -p $O
for v in base gdiag1 gdiag2 gdiag3; do
  L=""; [ $v != base ] && L=build_variants/$v/libtlod.so
  echo "$v fc   $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py 2>/dev/null)"
  echo "$v r101 $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py --r101 2>/dev/null)"
done
