# Round-6 validation of the committed tree: GPU tests of the given files (-m gpu), then
# __graft_entry__.smoke() when asked.  usage: bash tools/gpu/r6_validate.sh OUTDIR smoke|nosmoke files...
set -e
O=$1; S=$2; shift 2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
if [ "$S" = smoke ]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
