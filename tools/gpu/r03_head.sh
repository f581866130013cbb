# Round-3 lease: ResNet101 RoI head on the split-bf16 GEMM vs hipBLASLt fp32
# (TLOD_LINEAR_MATH=f32) — R101 / ATF / MAF step tests, bench A/B for DAF-R101 and ATF-R101.
# usage: bash tools/gpu/r03_head.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_resnet_gpu.py tests/test_atf_step_gpu.py tests/test_maf_step_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for r in 1 2; do
  for m in f32 bf16x6; do
    for cfg in "daf res101" "atf res101"; do
      set -- $cfg
      TLOD_LINEAR_MATH=$m timeout -k 10 400 python3 bench.py --method $1 --net $2 --steps 6 --warmup 2 --cpu-baseline-steps 0 > $O/b_${1}_${m}_${r}.json 2> $O/b_${1}_${m}_${r}.err
      echo "$m $cfg r$r: $(python3 -c "import json;d=json.load(open('$O/b_${1}_${m}_${r}.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
