# Small-GEMM tile A/B: the layout tests under each variant, bench_gemm (--da and the fc
# shapes) and DAF-VGG16.  usage: bash tools/gpu/r6_gsmall_ab.sh OUTDIR ROUNDS VARIANT...
set -e
O=$1; R=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in "$@"; do
  TLOD_LIB=build_variants/$v/libtlod.so timeout -k 10 300 python3 -m pytest tests/test_linear_gpu.py -q -x -k "layouts" --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  echo "tests $v: $(tail -1 $O/t_$v.log)"
done
for r in $(seq 1 $R); do
  for lab in new "$@"; do
    if [ $lab = new ]; then L=""; else L="TLOD_LIB=build_variants/$lab/libtlod.so"; fi
    env $L timeout -k 10 120 python3 tools/bench_gemm.py --da --no-torch > $O/g_$lab.$r.json 2>/dev/null
    env $L timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > $O/b_$lab.$r.json 2>/dev/null
    echo "$lab r$r: $(python3 -c "import json;d=json.load(open('$O/b_$lab.$r.json'));g=json.load(open('$O/g_$lab.$r.json'));print(d['value'], {k:v['ms'] for k,v in g.items()})")"
  done
done
