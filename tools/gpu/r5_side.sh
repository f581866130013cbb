# weight-gradient reduces on a side stream (TLOD_WGRAD_SIDE=1) vs in line (0)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_optim_gpu.py tests/test_conv_bs_gpu.py tests/test_dist_gpu.py tests/test_daf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    TLOD_WGRAD_SIDE=$v timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_WGRAD_SIDE=$v timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "side=$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
for v in 1 0; do
  TLOD_WGRAD_SIDE=$v timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.json 2>/dev/null
  echo "side=$v atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.json'))['value'])")"
done
