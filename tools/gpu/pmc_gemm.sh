# Clock / MFMA-busy / LDS counters of the head GEMM kernel (gemm_bs_kernel on fc6 / fc7
# forward, dgrad and wgrad at R = 556).  usage: bash tools/gpu/pmc_gemm.sh OUTDIR
set -e
O=$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- python3 tools/bench_gemm.py > $O/p1.out 2> $O/p1.err
python3 tools/pmc_kernel.py $O/p1 gemm > $O/p1.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/p2 -o run -- python3 tools/bench_gemm.py > $O/p2.out 2> $O/p2.err
python3 tools/pmc_kernel.py $O/p2 gemm > $O/p2.txt
cat $O/p1.txt $O/p2.txt
