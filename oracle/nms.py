"""Oracle: greedy NMS with the reference's CUDA-kernel semantics (test infrastructure only).

lib/model/nms/src/nms_cuda_kernel.cu:41-85 builds, for every pair (i < j) of the
score-sorted input, the bit ``devIoU(box_i, box_j) > thresh`` (devIoU :31-39, "+1" pixel
areas, strict >); the host loop :131-144 then keeps box i iff no earlier *kept* box set
its bit.  That is exactly the greedy scan below.  NOTE: the reference's numpy fallback
(nms_cpu.py:23-24 uses np.maximum for xx2/yy2) is a bug and is NOT restated.
"""
import numpy as np

from .boxes import iou_pair_cuda


def nms(dets, thresh, max_keep=None):
    """dets: (N, >=4) float32, already sorted by score (desc).  Returns int32 keep indices.

    ``max_keep`` truncates like the caller's ``keep[:post_nms_topN]``
    (proposal_layer.py:151-152) — the first ``max_keep`` survivors are identical.
    """
    dets = np.asarray(dets, dtype=np.float32)
    n = dets.shape[0]
    if n == 0:
        return np.zeros((0,), np.int32)  # nms_wrapper.py:15-16 returns []
    boxes = dets[:, :4]
    thr = np.float32(thresh)
    removed = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        if max_keep is not None and len(keep) >= max_keep:
            break
        if i + 1 < n:
            removed[i + 1:] |= iou_pair_cuda(boxes[i], boxes[i + 1:]) > thr
    return np.asarray(keep, dtype=np.int32)
