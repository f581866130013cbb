set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu/profile_r101.sh $O/prof
python3 tools/kstats.py $O/prof/daf/run_kernel_stats.csv 7 > $O/daf_per_step.txt 2>/dev/null || true
python3 tools/kstats.py $O/prof/atf/run_kernel_stats.csv 7 > $O/atf_per_step.txt 2>/dev/null || true
timeout -k 10 300 python3 tools/host_time.py 10 res101 daf > $O/host_daf.txt 2>&1
timeout -k 10 300 python3 tools/host_time.py 5 res101 atf > $O/host_atf.txt 2>&1
cat $O/host_daf.txt $O/host_atf.txt
