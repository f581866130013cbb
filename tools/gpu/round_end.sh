# Round end: full GPU test suite, smoke, then the round profile (tools/gpu/profile.sh).
# usage: bash tools/gpu/round_end.sh OUTDIR
set -e
cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
bash tools/gpu/profile.sh $O/prof $O/P
