# RoI head entry: tests, then DAF-R101 / ATF-R101 A/B (TLOD_ROI_HEAD_ENTRY=0/1)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_resnet_gpu.py tests/test_atf_step_gpu.py tests/test_maf_step_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for e in 1 0; do
    TLOD_ROI_HEAD_ENTRY=$e timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/daf.$e.$r.json 2>/dev/null
    TLOD_ROI_HEAD_ENTRY=$e timeout -k 10 300 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$e.$r.json 2>/dev/null
    echo "entry=$e r$r daf $(python3 -c "import json;print(json.load(open('$O/daf.$e.$r.json'))['value'])") atf $(python3 -c "import json;print(json.load(open('$O/atf.$e.$r.json'))['value'])")"
  done
done
