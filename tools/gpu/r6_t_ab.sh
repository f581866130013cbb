# tests of the given files, then bench A/B vs a variant on the given configs.
# usage: bash tools/gpu/r6_t_ab.sh OUTDIR VARIANT ROUNDS "tests..." "cfg" ...
set -e
O=$1; V=$2; R=$3; T=$4; shift 4
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 800 python3 -u -m pytest $T -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/r6_ab.sh $O/ab $R $V "$@"
