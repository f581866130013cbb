# Round-3 lease: rounding probe + bench A/B over the commits between r01 and HEAD.
# usage: bash tools/gpu/r03_bisect.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 tools/probe/mfma_round > $O/mfma_round.txt 2>&1
tail -25 $O/mfma_round.txt
timeout -k 10 1000 bash tools/gpu/ab.sh $O/ab 2 "r01=build_variants/r01" "cc6aa4f=build_variants/cc6aa4f" "cda15e5=build_variants/cda15e5" "r02end=build_variants/35d2ef2" "head=build_variants/head" "new=." > $O/ab.txt 2>&1
cat $O/ab.txt
