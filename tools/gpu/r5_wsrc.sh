# head conv weight gradients straight into their slots: tests + R101 / ATF lines
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_resnet_gpu.py tests/test_atf_step_gpu.py tests/test_maf_step_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.json 2>/dev/null
timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.json 2>/dev/null
echo "r101 $(python3 -c "import json;print(json.load(open('$O/r101.json'))['value'])") atf $(python3 -c "import json;print(json.load(open('$O/atf.json'))['value'])")"
timeout -k 10 200 python3 tools/arena_copies.py res101 daf 2>&1 | grep -v amdgpu | head -12
