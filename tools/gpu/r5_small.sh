# 1x1 Cout<=4 streaming conv (new) vs F.linear on a channels-last copy (old, TLOD_AB_SMALLCONV=0)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_conv_small_gpu.py tests/test_daf_step_gpu.py tests/test_atf_step_gpu.py tests/test_maf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    TLOD_AB_SMALLCONV=$v timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.$r.json 2>/dev/null
    TLOD_AB_SMALLCONV=$v timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 > $O/daf.$v.$r.json 2>/dev/null
    echo "new=$v r$r atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.$r.json'))['value'])") daf $(python3 -c "import json;print(json.load(open('$O/daf.$v.$r.json'))['value'])")"
  done
done
