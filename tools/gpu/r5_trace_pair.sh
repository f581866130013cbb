# kernel timeline of the conv3_3 dgrad / wgrad pair on two streams, plus GEMM A/B
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_conv.py --math bf16x6 --iters 10 > $O/kt.out 2> $O/kt.err
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_gemm.py > $O/gnew.$r.json; echo "new  $(cat $O/gnew.$r.json)"
  TLOD_LIB=build_variants/base/libtlod.so timeout -k 10 120 python3 tools/bench_gemm.py > $O/gbase.$r.json; echo "base $(cat $O/gbase.$r.json)"
done
