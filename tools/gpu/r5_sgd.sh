# fused SGD pack microbench A/B with kernel stats
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in 1 0; do TLOD_SGD_PACK=$v timeout -k 10 120 python3 tools/bench_sgd.py; done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0; do
  TLOD_SGD_PACK=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python3 tools/bench_sgd.py > /dev/null 2>&1
  f=$(find $O/p$v -name '*kernel_stats.csv' | head -1); echo "pack=$v"; cut -d, -f1-8 $f | head -8
done
