# head-entry backward gather: per-sample bin rows from the geometry pass (new) vs per-tap index
# arithmetic (rhead)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in new rhead; do
    L=""; [ $v != new ] && L=build_variants/$v/libtlod.so
    TLOD_LIB=$L timeout -k 10 400 python3 bench.py --method atf --net res101 --steps 8 --warmup 3 --cpu-baseline-steps 0 > $O/atf.$v.$r.json 2>/dev/null
    TLOD_LIB=$L timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "$v r$r atf $(python3 -c "import json;print(json.load(open('$O/atf.$v.$r.json'))['value'])") vgg $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --method atf --net res101 --steps 3 --warmup 1 --cpu-baseline-steps 0 > /dev/null 2>&1
grep -E "rbg|roi_align|nhwc" $O/prof/run_kernel_stats.csv | cut -d, -f1-4
