# Round-2 profile at HEAD: kernel stats of the bench command, PMC HBM traffic passes,
# the conv3_3 backward microbench (+ its kernel stats), a 2-rank gloo rehearsal of the
# multi-GPU bench path, and the default bench line (with the CPU baseline).
set -e
O=gpurun_out/r02
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
rm -rf $O/stats $O/fetch $O/write $O/conv33_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/bench_rocprof.json 2> $O/stats.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > /dev/null 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > /dev/null 2> $O/write.err
python3 tools/pmc_traffic.py $O/fetch $O/write 13 $O/traffic.json > /dev/null
timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 > $O/conv33.json 2> $O/conv33.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conv33_stats -o run -- python3 tools/bench_conv.py --math bf16x6 > $O/conv33_rocprof.json 2> $O/conv33_stats.err
TLOD_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 4 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
mkdir -p profiles/r02 && cp $O/traffic.json profiles/r02/traffic.json
timeout -k 10 600 python3 bench.py > $O/bench_line.json 2> $O/bench_line.err
cat $O/bench_line.json | cut -c 1-600
cat $O/conv33.json
cat $O/bench_gloo2.json | cut -c 1-300
