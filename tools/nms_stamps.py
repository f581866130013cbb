"""Per-block stamps of the NMS greedy scan (diagnostic; needs a libtlod built with the
stamped scan, TLOD_LIB=...).  Prints per block: cycles from block start to wave 0's
resolution, to thread 64's far-column OR, to the barrier, and to the next block start."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "transfer-learning-library-for-object-detection_amd"))
from bench_nms import anchors_image  # noqa: E402
from tlod import _lib  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.lib()
rng = np.random.default_rng(0)
boxes = anchors_image(rng)
s = rng.permutation(len(boxes)).astype(np.float32) / len(boxes)
order = np.argsort(-s, kind="stable")
dets = np.concatenate([boxes[order], s[order, None]], 1).astype(np.float32)
n, mk = 12000, 2000
d = torch.from_numpy(dets[:n]).to(dev).contiguous()
keep = torch.empty(n, dtype=torch.int32, device=dev)
num = torch.empty(1, dtype=torch.int32, device=dev)
ws = torch.empty(L.tlod_nms_workspace_bytes(n), dtype=torch.uint8, device=dev)
for _ in range(3):
    _lib.check(L.tlod_nms_f32(_lib.ptr(d), n, 5, 0.7, mk, _lib.ptr(keep), _lib.ptr(num),
                              _lib.ptr(ws), ws.numel(), _lib.stream_of(d)), "nms")
torch.cuda.synchronize()
st = (ctypes.c_ulonglong * (20 * 512))()
assert L.tlod_nms_debug_stamps(st) == 0
a = np.array(st, dtype=np.int64).reshape(512, 20)
nb = int((a[:, 0] > 0).sum())
a = a[:nb]
t0 = a[0, 0]
print("blocks", nb, "total cycles", a[-1, 2] - a[0, 0])
for b in list(range(0, min(nb, 8))) + list(range(max(8, nb - 4), nb)):
    nxt = a[b + 1, 0] - a[b, 0] if b + 1 < nb else 0
    pre = " ".join(f"{v:5d}" for v in (a[b, 4:20] - a[b, 0]))
    print(f"b={b:3d} resolve {a[b,1]-a[b,0]:5d} barrier {a[b,2]-a[b,0]:5d} next {nxt:5d} | "
          f"pre-barrier per wave: {pre}")
dt = np.diff(a[:, 0])
print("median per block", int(np.median(dt)), "resolve", int(np.median(a[:, 1] - a[:, 0])),
      "barrier", int(np.median(a[:, 2] - a[:, 0])), "pre-barrier per wave",
      [int(v) for v in np.median(a[:, 4:20] - a[:, :1], 0)])
