# Round profile of HEAD: rocprofv3 kernel stats of the bench command, PMC HBM traffic passes
# (FETCH_SIZE, WRITE_SIZE: separate runs; 14 steps per bench run = 3 warmup + 1 launch-count probe + 10 timed), the conv3_3 backward microbench and its kernel
# stats, per-shape conv timings.  usage: bash tools/gpu/profile.sh OUTDIR [PROFILE_DIR]
set -e
O=$1; P=${2:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
rm -rf $O/stats $O/fetch $O/write $O/conv33_stats
B="python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/bench_rocprof.json 2> $O/stats.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > /dev/null 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > /dev/null 2> $O/write.err
python3 tools/pmc_traffic.py $O/fetch $O/write 14 $O/traffic.json > /dev/null || true
timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 > $O/conv33.json 2> $O/conv33.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/conv33_stats -o run -- python3 tools/bench_conv.py --math bf16x6 > $O/conv33_rocprof.json 2> $O/conv33_stats.err
TLOD_BENCH_SHAPES=1 timeout -k 10 200 $B > $O/bench_shapes.json 2> $O/bench_shapes.err
# BASELINE configs 3-5 (per GPU): DAF ResNet101, MAF VGG16, ATF ResNet101 (21 classes)
for cfg in "daf res101" "maf vgg16" "atf res101"; do
  set -- $cfg
  timeout -k 10 400 python3 bench.py --method $1 --net $2 --steps 10 --warmup 3 --cpu-baseline-steps 0 \
    > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err
done
if [ -n "$P" ]; then
  mkdir -p $P
  cp $O/traffic.json $P/traffic.json
  cp $O/stats/run_kernel_stats.csv $P/bench_kernel_stats.csv
  cp $O/stats/run_domain_stats.csv $P/bench_domain_stats.csv 2>/dev/null || true
  cp $O/conv33.json $P/conv33_bwd.json
  cp $O/conv33_stats/run_kernel_stats.csv $P/conv33_kernel_stats.csv
  cp $O/bench_rocprof.json $P/bench_line_rocprof.json
  cp $O/bench_shapes.err $P/bench_conv_shapes.txt
  for f in $O/bench_daf_res101.json $O/bench_maf_vgg16.json $O/bench_atf_res101.json; do
    cp $f $P/
  done
fi
cat $O/conv33.json
