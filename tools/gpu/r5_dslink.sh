# ResNet head: downsample shortcut gradient via the link into conv1 dgrad (new) vs autograd sum (old)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_resnet_gpu.py tests/test_atf_step_gpu.py tests/test_daf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    TLOD_AB_DSLINK=$v timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.$r.json 2>/dev/null
    TLOD_AB_DSLINK=$v timeout -k 10 400 python3 bench.py --method daf --net res101 --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "new=$v r$r atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.$r.json'))['value'])") daf-r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
