set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/a.$r.json; cat $O/a.$r.json
  TLOD_CONV_KSPLIT_MAX=1 timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/b.$r.json; cat $O/b.$r.json
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TLOD_CONV_KSPLIT_MAX=1 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_conv.py --math bf16x6 --iters 10 > $O/kt.out 2> $O/kt.err
