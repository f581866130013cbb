# Full GPU test suite + smoke, then bench
mkdir -p gpurun_out/full
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/full/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/full/pytest.log
grep -E "FAIL|device error" gpurun_out/full/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 && tail -1 gpurun_out/full/smoke.log
