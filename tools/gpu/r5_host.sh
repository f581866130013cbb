# host-side launch overhead: raw stream accessor (new) vs torch.cuda.current_stream (old)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_resnet_gpu.py tests/test_daf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 0 1; do
    TLOD_AB_OLDSTREAM=$v timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_AB_OLDSTREAM=$v timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "old=$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
TLOD_AB_OLDSTREAM=0 timeout -k 10 300 python3 tools/host_time.py 10 res101 daf 2>&1 | grep -v amdgpu | tail -2
TLOD_AB_OLDSTREAM=1 timeout -k 10 300 python3 tools/host_time.py 10 res101 daf 2>&1 | grep -v amdgpu | tail -2
