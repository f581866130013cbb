# conv3_3 backward with dgrad / wgrad on two streams, with and without split-K tails.
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/pair.$r.json; cat $O/pair.$r.json
  TLOD_CONV_KSPLIT_MAX=1 timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/nosplit.$r.json; cat $O/nosplit.$r.json
done
