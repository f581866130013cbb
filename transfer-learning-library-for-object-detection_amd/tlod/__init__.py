"""tlod — MI355X-native (gfx950) hot path of the domain-adaptive Faster R-CNN training
step (DAF / MAF / ATF) of Transfer-Learning-Library-for-Object-Detection.

Kernels live in libtlod.so (csrc/, C ABI in include/tlod.h); this package is the host
side that mirrors the reference's plugin surface (lib/model/{nms,roi_align,roi_pooling,
rpn,faster_rcnn}, lib/DAF, lib/MAF, lib/ATF) on top of that ABI.
"""
__version__ = "0.1.0"
