# Kernel stats of DAF-R101 and ATF-R101 (rocprofv3), GPU busy fraction.
# usage: bash tools/gpu/profile_r101.sh OUTDIR
set -e
O=$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
for m in daf atf; do
  B="python3 bench.py --method $m --net res101 --steps 5 --warmup 2 --cpu-baseline-steps 0"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- $B > $O/$m.json 2> $O/$m.err
  python3 tools/gpu_busy.py $O/$m/run_kernel_trace.csv 0.3 | head -3
done
