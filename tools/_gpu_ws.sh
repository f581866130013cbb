# Persistent warp-specialized split-bf16 forward: parity under TLOD_CONV_WS=1, A/B, stamps.
set -e
mkdir -p gpurun_out/ws
export PYTHONUNBUFFERED=1
TLOD_CONV_WS=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_bs_gpu.py tests/test_pool_gpu.py > gpurun_out/ws/tests1.log 2>&1 || { tail -30 gpurun_out/ws/tests1.log; exit 1; }
tail -1 gpurun_out/ws/tests1.log
for v in "TLOD_CONV_WS=0" "TLOD_CONV_WS=1" "TLOD_CONV_WS=1 TLOD_WS_PERSIST=1" "TLOD_CONV_WS=0" "TLOD_CONV_WS=1"; do
  echo "== $v"
  for shp in "" "--C 512 --H 75 --W 150" "--C 64 --H 300 --W 600"; do
    env $v timeout -k 10 120 python3 tools/bench_conv.py --math bf16x6 $shp | python3 -c "import json,sys;d=json.load(sys.stdin);print('  fwd %.4f dgrad %.4f wgrad %.4f'%(d['fwd_ms'],d['dgrad_ms'],d['wgrad_ms']))"
  done
done
