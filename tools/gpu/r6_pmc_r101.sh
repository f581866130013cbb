# PMC passes over the DAF-R101 bench (the 1x1 conv GEMMs and split-K reduces): clock / MFMA
# busy / waits, then FETCH_SIZE and WRITE_SIZE.  usage: bash tools/gpu/r6_pmc_r101.sh OUTDIR
set -e
O=$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
B="python3 bench.py --method daf --net res101 --steps 3 --warmup 2 --cpu-baseline-steps 0"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- $B > $O/p1.out 2> $O/p1.err
python3 tools/pmc_kernel.py $O/p1 conv_gemm > $O/p1.txt
python3 tools/pmc_kernel.py $O/p1 reduce >> $O/p1.txt
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run -- $B > $O/p2.out 2> $O/p2.err
python3 tools/pmc_kernel.py $O/p2 conv_gemm > $O/p2.txt
cat $O/p1.txt $O/p2.txt
