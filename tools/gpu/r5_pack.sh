# Weight packs written by the fused SGD: tests, then DAF-VGG16 / DAF-R101 A/B (TLOD_SGD_PACK=1/0)
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_optim_gpu.py tests/test_daf_step_gpu.py tests/test_resnet_gpu.py tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 1 0; do
    TLOD_SGD_PACK=$v timeout -k 10 300 python3 bench.py --cpu-baseline-steps 0 > $O/vgg.$v.$r.json 2>/dev/null
    TLOD_SGD_PACK=$v timeout -k 10 300 python3 bench.py --method daf --net res101 --cpu-baseline-steps 0 > $O/r101.$v.$r.json 2>/dev/null
    echo "pack=$v r$r vgg $(python3 -c "import json;print(json.load(open('$O/vgg.$v.$r.json'))['value'])") r101 $(python3 -c "import json;print(json.load(open('$O/r101.$v.$r.json'))['value'])")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --cpu-baseline-steps 0 > $O/prof.json 2>/dev/null
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/vgg_kernel_stats.csv \;
grep -E "sgd|pack" $O/vgg_kernel_stats.csv | cut -c1-160
