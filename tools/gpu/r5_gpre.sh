# GEMM one-slot loop with the half-way staging pinned (new) vs HEAD's loop (gbase), and the RoI
# head's fused backward (TLOD_HEAD_FUSE=1/0)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_linear_gpu.py tests/test_conv_bs_gpu.py tests/test_resnet_gpu.py tests/test_atf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new gbase; do
  L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
  echo "$v fc   $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py 2>/dev/null)"
  echo "$v r101 $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py --r101 2>/dev/null)"
done
for r in 1 2; do
  for v in new.1 new.0 gbase.0; do
    b=${v%.*}; f=${v#*.}
    L=""; [ $b != new ] && L=build_variants/$b/libtlod.so
    TLOD_HEAD_FUSE=$f TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_HEAD_FUSE=$f TLOD_LIB=$L timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
for v in new.1 new.0 gbase.0; do
  b=${v%.*}; f=${v#*.}
  L=""; [ $b != new ] && L=build_variants/$b/libtlod.so
  TLOD_HEAD_FUSE=$f TLOD_LIB=$L timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.json 2>/dev/null
  echo "$v atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.json'))['value'])")"
done
