# Round-6 profile capture at the final tree, in two parts (each one gpurun call):
#   part a: bench kernel stats + PMC traffic + conv3_3 microbench + per-shape conv TF +
#           configs 3-5 (tools/gpu/profile.sh -> profiles/r06);
#   part b: the ResNet101 kernel stats, the conv3 PMC passes (clock / MFMA busy / LDS), the
#           default bench line.
# usage: bash tools/gpu/r6_capture.sh OUTDIR a|b
set -e
O=$1; PART=$2
P=profiles/r06
mkdir -p $O $P
if [ "$PART" = a ]; then
  bash tools/gpu/profile.sh $O/prof $P
  python3 tools/kstats.py $P/bench_kernel_stats.csv 14 > $P/bench_kernel_per_step.txt 2>/dev/null || true
else
  bash tools/gpu/profile_r101.sh $O/r101 > $O/r101_busy.txt 2>&1 || true
  for m in daf atf; do
    cp $O/r101/$m/run_kernel_stats.csv $P/${m}_res101_kernel_stats.csv || true
    python3 tools/kstats.py $O/r101/$m/run_kernel_stats.csv 7 > $P/${m}_res101_kernel_per_step.txt 2>/dev/null || true
  done
  bash tools/gpu/pmc_conv.sh $O/pmc > /dev/null 2>&1 || true
  cp $O/pmc/p1.txt $P/pmc_conv3_3_mfma_busy.txt || true
  cp $O/pmc/p2.txt $P/pmc_conv3_3_lds.txt || true
  timeout -k 10 400 python3 bench.py > $P/bench_line.json 2> $O/bench_line.err
  cat $P/bench_line.json
fi
