# Round-3 lease: ATF-ResNet101 (config 5) step breakdown: host enqueue time, rocprofv3 kernel
# stats, GPU busy fraction.  usage: bash tools/gpu/r03_atf.sh OUTDIR
set -e
O=$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 tools/host_time.py 6 res101 atf > $O/host.txt 2>&1
tail -1 $O/host.txt
B="python3 bench.py --method atf --net res101 --steps 5 --warmup 2 --cpu-baseline-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/rocprof.json 2> $O/stats.err
python3 tools/gpu_busy.py $O/stats/run_kernel_trace.csv 0.5 | head -8
