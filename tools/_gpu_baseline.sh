# Baseline at round start: headline bench + conv3_3 microbench.
set -e
mkdir -p gpurun_out/base
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > gpurun_out/base/bench.json 2> gpurun_out/base/bench.err
timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 > gpurun_out/base/conv33.json 2>&1
cat gpurun_out/base/bench.json gpurun_out/base/conv33.json
