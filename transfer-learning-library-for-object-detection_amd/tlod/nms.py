"""Drop-in for ``model.nms.nms_wrapper.nms`` (lib/model/nms/nms_wrapper.py:13-21).

Same signature and return convention: int32 indices into the (score-sorted) ``dets``,
``[]`` for an empty input.  The work runs in libtlod's on-device NMS (mask + greedy scan,
include/tlod.h ``tlod_nms_f32``); there is no host round trip and no CPU fallback.
"""
import torch

from . import _lib


def nms(dets, thresh, force_cpu=False, max_keep=0):
    """dets: (N, 5) CUDA float32 [x1, y1, x2, y2, score], sorted by score descending.

    ``force_cpu=True`` selected the reference's numpy fallback, whose IoU is wrong
    (nms_cpu.py:23-24 uses np.maximum for xx2/yy2); this path does not reproduce it.
    ``max_keep`` (extension) stops after that many survivors.
    """
    if dets.shape[0] == 0:
        return []
    if force_cpu:
        raise NotImplementedError("tlod.nms: no CPU NMS (the reference's nms_cpu is buggy, "
                                  "nms_cpu.py:23-24); pass CUDA tensors")
    _lib.require_cuda(dets)
    d = dets.contiguous().float()
    n, dim = d.shape
    L = _lib.lib()
    keep = torch.empty(n, dtype=torch.int32, device=d.device)
    num = torch.empty(1, dtype=torch.int32, device=d.device)
    ws = _lib.workspace(L.tlod_nms_workspace_bytes(n), d.device, "nms")
    _lib.check(L.tlod_nms_f32(_lib.ptr(d), n, dim, float(thresh), int(max_keep), _lib.ptr(keep),
                              _lib.ptr(num), _lib.ptr(ws), ws.numel(), _lib.stream_of(d)), "nms")
    return keep[: int(num.item())]  # host read of the count, as nms_gpu.py:11 does
