export PYTHONUNBUFFERED=1
for v in "X=1" "TLOD_CONV_MATH=f32" "TLOD_LINEAR_MATH=f32" "TLOD_CONV_MATH=f32 TLOD_LINEAR_MATH=f32" "TLOD_WGRAD_MATH=f32" "TLOD_FUSED_LOSSES=0"; do
  echo "== $v"
  env $v timeout -k 10 300 python3 tools/scratch/diag_frcnn_inter.py 2>&1 | grep -v amdgpu | grep "RCNN_base.10\|RCNN_cls\|base    fwd\|base    grad"
done
