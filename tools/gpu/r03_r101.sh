# Round-3 lease: DAF-ResNet101 step breakdown (rocprofv3 kernel stats + per-shape conv TF).
# usage: bash tools/gpu/r03_r101.sh OUTDIR
set -e
O=$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
B="python3 bench.py --net res101 --steps 10 --warmup 3 --cpu-baseline-steps 0"
TLOD_BENCH_SHAPES=1 timeout -k 10 300 $B > $O/shapes.json 2> $O/shapes.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/rocprof.json 2> $O/stats.err
