# Round-3 lease: MFMA rounding probe, split-bf16 conv tests on the working tree, bench A/B
# r01 / committed HEAD / working tree, bench lines of configs 3-5 (working tree).
# usage: bash tools/gpu/r03_ab.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 tools/probe/mfma_round > $O/mfma_round.txt 2>&1
echo probe done
timeout -k 10 600 python -u -m pytest tests/test_conv_bs_gpu.py tests/test_pool_gpu.py tests/test_maf_step_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "r01=build_variants/r01" "head=build_variants/head" "new=." > $O/ab.txt 2>&1
cat $O/ab.txt
for cfg in "--net res101" "--method maf" "--method atf"; do
  tag=$(echo $cfg | tr -d '-' | tr ' ' '_')
  timeout -k 10 300 python3 bench.py $cfg --cpu-baseline-steps 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  echo "$cfg: $(python3 -c "import json;d=json.load(open('$O/bench_$tag.json'));print(d['value'], d['ms_per_step'])")"
done
