# the GPU tests from test_eval_gpu on (alphabetical), smoke, bench
set -e
O=$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests/test_eval_gpu.py tests/test_frcnn_gpu.py tests/test_golden.py tests/test_linear_gpu.py tests/test_losses_gpu.py tests/test_maf_step_gpu.py tests/test_ops_gpu.py tests/test_optim_gpu.py tests/test_pool_gpu.py tests/test_resnet_gpu.py tests/test_rpn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
