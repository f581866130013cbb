# Round-3 lease: full GPU suite, then the round profile of the tree (profiles/r03) and a
# bench A/B against the committed round-2 HEAD.  usage: bash tools/gpu/r03_full.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -2 $O/pytest.log
timeout -k 10 900 bash tools/gpu/profile.sh $O/prof profiles/r03 > $O/prof.txt 2>&1
echo profile done
timeout -k 10 600 bash tools/gpu/ab.sh $O/ab 2 "head=build_variants/head" "new=." > $O/ab.txt 2>&1
cat $O/ab.txt
