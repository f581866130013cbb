# conv kernels' staging pinned (1x1 / 3x3 im2col wgrad, plain split-bf16 fwd) vs HEAD (cbase)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_conv_bs_gpu.py tests/test_resnet_gpu.py tests/test_maf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new cbase; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    echo "$v x $(TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_1x1.py 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(json.load(sys.stdin)["total_ms"])')"
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
