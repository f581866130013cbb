# Final-tree check on one GPU: the full GPU test suite, smoke(), then the default bench line.
# usage: bash tools/gpu/validate.sh OUTDIR
set -e
O=${1:-gpurun_out/validate}
rm -rf $O; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
