set -e
mkdir -p gpurun_out/acc
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 tools/scratch/diag_fwd_layers.py 2>&1 | grep layer
timeout -k 10 200 python3 tools/scratch/conv_err.py 2>&1 | grep -v amdgpu
timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > gpurun_out/acc/bench.json 2>gpurun_out/acc/bench.err
python3 -c "import json;d=json.load(open('gpurun_out/acc/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_frcnn_gpu.py tests/test_daf_step_gpu.py tests/test_conv_bs_gpu.py tests/test_linear_gpu.py > gpurun_out/acc/pytest.log 2>&1 || true
grep -E "worst|passed|failed|FAIL" gpurun_out/acc/pytest.log | head -20
