set -e
mkdir -p gpurun_out/diag
export PYTHONUNBUFFERED=1
run() { env "$@" timeout -k 10 200 python3 tools/scratch/diag_daf_grads.py 192 320 0 2>&1 | grep worst; }
run DIAG_TAG=default
run DIAG_TAG=losses_torch TLOD_FUSED_LOSSES=0
run DIAG_TAG=act_torch TLOD_FUSED_ACT=0
run DIAG_TAG=linear_f32 TLOD_LINEAR_MATH=f32
run DIAG_TAG=conv_f32 TLOD_CONV_MATH=f32
run DIAG_TAG=all_f32 TLOD_CONV_MATH=f32 TLOD_LINEAR_MATH=f32 TLOD_FUSED_LOSSES=0 TLOD_FUSED_ACT=0
run DIAG_TAG=unbatched DIAG_UNBATCHED=1
