# Full GPU test suite at HEAD defaults, then bench A/B of env variants (args).
set -e
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/suite.log 2>&1 || { tail -40 gpurun_out/ab/suite.log; exit 1; }
tail -2 gpurun_out/ab/suite.log
bash tools/_gpu_ab_bench.sh "$@"
