set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
for w in 32 16 64; do
  timeout -k 10 300 python3 tools/overlap_probe.py --steps 5 --contend --contend-wgs $w > $O/contend_$w.json 2> $O/contend_$w.err
  python3 -c "import json;d=json.load(open('$O/contend_$w.json'));print($w, d['contention'], d['prediction']['153GBps'])"
done
