# Round 5: ws conv staging layout — GPU conv tests, conv3_3 microbench A/B vs a baseline
# build (build_variants/base), LDS/MFMA PMC passes.  usage: bash tools/gpu/r5_ws.sh OUTDIR
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests/test_conv_bs_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/new.$r.json
  TLOD_LIB=build_variants/base/libtlod.so timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 --iters 40 > $O/base.$r.json
  echo "new  $(cat $O/new.$r.json)"; echo "base $(cat $O/base.$r.json)"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="python3 tools/bench_conv.py --math bf16x6 --iters 20"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $O/p2 -o run -- $C > $O/p2.out 2> $O/p2.err
python3 tools/pmc_kernel.py $O/p2 > $O/p2.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/p1 -o run -- $C > $O/p1.out 2> $O/p1.err
python3 tools/pmc_kernel.py $O/p1 > $O/p1.txt
head -4 $O/p1.txt $O/p2.txt
