# Targeted GPU tests + bench; args: pytest selection
set -e
mkdir -p gpurun_out/check
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $* > gpurun_out/check/pytest.log 2>&1 || { tail -60 gpurun_out/check/pytest.log; exit 1; }
tail -5 gpurun_out/check/pytest.log
timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err
cut -c 1-400 gpurun_out/check/bench.json
