# GEMM epilogue A/B: tests of the GEMM users, then bench_gemm (VGG head and ATF shapes) for the
# tree vs build_variants/gemm_old.  usage: bash tools/gpu/r6_gemm_ab.sh OUTDIR
set -e
O=${1:-gpurun_out/r6ga}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_linear_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for v in new old; do
    if [ $v = new ]; then L=""; else L="TLOD_LIB=build_variants/gemm_old/libtlod.so"; fi
    env $L timeout -k 10 120 python3 tools/bench_gemm.py --no-torch > $O/vgg_$v$i.json
    env $L timeout -k 10 200 python3 tools/bench_gemm.py --atf --no-torch > $O/atf_$v$i.json
  done
done
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
for kind in ("vgg", "atf"):
    a = [json.load(open(f"{O}/{kind}_new{i}.json")) for i in (1, 2)]
    b = [json.load(open(f"{O}/{kind}_old{i}.json")) for i in (1, 2)]
    for k in a[0]:
        na = min(x[k]["ms"] for x in a); nb = min(x[k]["ms"] for x in b)
        print(f"{kind} {k:20s} new {na:7.3f}  old {nb:7.3f}  {100*(na/nb-1):+5.1f}%")
PY
