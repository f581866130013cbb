# NMS mask: division-free exact IoU threshold + per-box areas (new) vs division (nmsv3)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_rpn_gpu.py -x -q -k "nms or proposal" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new nmsv3 new nmsv3; do
  L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
  echo "== $v"; TLOD_LIB=$L timeout -k 10 120 python3 tools/bench_nms.py 100
done
for r in 1 2; do
  for v in new nmsv3; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --cpu-baseline-steps 0 > $O/daf.$v.$r.json 2>/dev/null
    echo "$v r$r daf $(python3 -c "import json;print(json.load(open('$O/daf.$v.$r.json'))['value'])")"
  done
done
