# Round profile: kernel stats of the bench command, PMC HBM traffic passes, and the bench
# line with the CPU baseline.  Writes gpurun_out/r01/.
set -e
mkdir -p gpurun_out/r01
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r01
rm -rf $O/stats $O/fetch $O/write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/bench_rocprof.json 2> $O/stats.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > /dev/null 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > /dev/null 2> $O/write.err
timeout -k 10 400 python3 bench.py > $O/bench_line.json 2> $O/bench_line.err
ls -R $O | head -30
