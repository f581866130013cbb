# Round-3 baseline lease: MFMA rounding probe, r01-vs-HEAD bench A/B, HEAD profile into
# profiles/r03, bench lines of configs 3-5.  usage: bash tools/gpu/r03_base.sh
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 tools/probe/mfma_round > $O/mfma_round.txt 2>&1
echo probe done
timeout -k 10 900 bash tools/gpu/ab.sh $O/ab 3 "r01=build_variants/r01" "head=." > $O/ab.txt 2>&1
cat $O/ab.txt
timeout -k 10 900 bash tools/gpu/profile.sh $O/prof profiles/r03 > $O/prof.txt 2>&1
echo profile done
for cfg in "--net res101" "--method maf" "--method atf" "--net res101 --method maf" "--net res101 --method atf"; do
  tag=$(echo $cfg | tr -d '-' | tr ' ' '_')
  timeout -k 10 300 python3 bench.py $cfg --cpu-baseline-steps 0 > $O/bench_$tag.json 2> $O/bench_$tag.err
  echo "$cfg: $(python3 -c "import json;d=json.load(open('$O/bench_$tag.json'));print(d['value'], d['ms_per_step'])")"
done
