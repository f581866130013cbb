# Kernel stats of one bench config for this tree and a variant.  usage: r6_kstat.sh OUT VARIANT method net
set -e
O=$1; V=$2; M=$3; N=$4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for lab in new $([ "$V" = - ] || echo $V); do
  if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$V/libtlod.so"; fi
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$lab -o run -- python3 bench.py --method $M --net $N --steps 5 --warmup 2 --cpu-baseline-steps 0 > $O/$lab.json 2> $O/$lab.err
  python3 tools/kstats.py $O/$lab/run_kernel_stats.csv 7 > $O/$lab.txt 2>/dev/null || python3 -c "
import csv
rows=sorted(csv.DictReader(open('$O/$lab/run_kernel_stats.csv')), key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print('%9.3f ms/step %7.1f calls/step %s' % (float(r['TotalDurationNs'])/7e6, int(r['Calls'])/7, r['Name'][:100]))
" > $O/$lab.txt
  echo "== $lab"; head -25 $O/$lab.txt
done
