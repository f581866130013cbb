# Round-3 lease: split-bf16 conv tests + bench A/B of the per-k-step product sums (KSUM16).
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_bs_gpu.py tests/test_pool_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "ksum=." "ksum0=.:TLOD_LIB=build_variants/ksum0/libtlod.so" > $O/ab.txt 2>&1
cat $O/ab.txt
