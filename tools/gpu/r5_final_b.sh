# Round-5 profile capture: bench kernel stats + PMC traffic + conv3_3 microbench + configs 3-5
# (tools/gpu/profile.sh -> profiles/r05), then DAF-R101 / ATF-R101 kernel stats.
set -e
O=$1
bash tools/gpu/profile.sh $O/prof profiles/r05
bash tools/gpu/profile_r101.sh $O/r101 > $O/r101_busy.txt 2>&1 || true
for m in daf atf; do
  cp $O/r101/$m/run_kernel_stats.csv profiles/r05/${m}_res101_kernel_stats.csv
  python3 tools/kstats.py $O/r101/$m/run_kernel_stats.csv 8 > profiles/r05/${m}_res101_kernel_per_step.txt 2>/dev/null || true
done
python3 tools/kstats.py profiles/r05/bench_kernel_stats.csv 14 > profiles/r05/bench_kernel_per_step.txt 2>/dev/null || true
cat $O/r101_busy.txt
