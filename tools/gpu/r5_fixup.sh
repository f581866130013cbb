# ws conv split-K fixup in the launch: conv tests, then A/B vs build_variants/nofix (HEAD conv.hip)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_conv_bs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new nofix; do
    L=""; [ $v = nofix ] && L=build_variants/nofix/libtlod.so
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/c33.$v.$r.json
    echo "$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])") c33 $(python3 -c "import json;d=json.load(open('$O/c33.$v.$r.json'));print(d['fwd_ms'],d['dgrad_ms'],d['wgrad_ms'])")"
  done
done
