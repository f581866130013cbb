set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
ls -R gpurun_out/prof | head -20
