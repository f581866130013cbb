# GEMM MFMA form A/B: default (16x16x32 paired planes, 1x1 OCC2), m2noocc, m0 (32x32x16)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_linear_gpu.py tests/test_conv_bs_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in def m2noocc m0; do
    L=""; [ $v != def ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_gemm.py > $O/g.$v.$r.json
    TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_1x1.py > $O/x.$v.$r.json 2>&1
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])") gemm $(python3 -c "import json;d=json.load(open('$O/g.$v.$r.json'));print(' '.join(f'{k}={v[\"ms\"]}' for k,v in d.items()))")"
  done
done
for v in def m0; do
  L=""; [ $v != def ] && L=build_variants/$v/libtlod.so
  TLOD_LIB=$L timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.json 2>/dev/null
  echo "$v atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.json'))['value'])")"
done
