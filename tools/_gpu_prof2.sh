set -e
mkdir -p gpurun_out/prof2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_daf_step_gpu.py > gpurun_out/prof2/pytest.log 2>&1 || { tail -30 gpurun_out/prof2/pytest.log; exit 1; }
tail -2 gpurun_out/prof2/pytest.log
rm -rf gpurun_out/prof2/stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/stats -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0 > gpurun_out/prof2/bench.json 2> gpurun_out/prof2/stats.err
f=$(find gpurun_out/prof2/stats -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["TotalDurationNs"])/1e6/13:8.3f} ms/step  {int(r["Calls"])/13:6.1f}/step  avg {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:110]}')
PY
