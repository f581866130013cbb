set -e
export PYTHONUNBUFFERED=1
timeout -k 10 200 python3 tools/scratch/diag_layer_bias.py 2>&1 | grep -v amdgpu | head -3
timeout -k 10 200 python3 tools/scratch/diag_fwd_layers.py 2>&1 | grep "layer 28"
timeout -k 10 300 python3 tools/scratch/diag_frcnn_inter.py 2>&1 | grep -v amdgpu | grep "RCNN\|base"
timeout -k 10 300 python3 tools/bench_conv.py --math bf16x6 2>&1 | grep -v amdgpu
