set -e
mkdir -p gpurun_out/calib
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/calib/*
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run -- python3 tools/calib_traffic.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/write -o run -- python3 tools/calib_traffic.py > /dev/null 2>&1
python3 - <<'PY'
import csv
for d, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    for r in csv.DictReader(open(f"gpurun_out/calib/{d}/run_counter_collection.csv")):
        if r["Counter_Name"] == c and ("conv_fwd_bs" in r["Kernel_Name"] or "conv_wgrad_bs" in r["Kernel_Name"] or "slab" in r["Kernel_Name"]):
            print(c, r["Kernel_Name"][:60], float(r["Counter_Value"]) / 1024.0, "MB")
PY
