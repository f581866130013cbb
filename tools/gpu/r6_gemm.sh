# ATF-R101 head GEMM study: timings of the layer4 shapes (R = 72192 rows) for the tile-order
# variants, then MFMA-busy / wait and FETCH_SIZE / WRITE_SIZE PMC passes of the default build.
# usage: bash tools/gpu/r6_gemm.sh OUTDIR
set -e
O=${1:-gpurun_out/r6g}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
G="python3 tools/bench_gemm.py --atf --no-torch"
for v in base gord1 gord2 base; do
  if [ $v = base ]; then L=""; else L="TLOD_LIB=build_variants/$v/libtlod.so"; fi
  env $L timeout -k 10 200 $G > $O/t_$v.json 2> $O/t_$v.err
  echo "$v $(cat $O/t_$v.json)"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- $G > $O/p1.out 2> $O/p1.err
python3 tools/pmc_kernel.py $O/p1 gemm > $O/p1.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run -- $G > $O/p2.out 2> $O/p2.err
python3 tools/pmc_kernel.py $O/p2 gemm > $O/p2.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/p3 -o run -- $G > $O/p3.out 2> $O/p3.err
python3 tools/pmc_kernel.py $O/p3 gemm > $O/p3.txt
cat $O/p1.txt $O/p2.txt $O/p3.txt
