"""CPU restatement ("oracle") of the reference's hot path — TEST INFRASTRUCTURE ONLY.

This package restates, in numpy float32/float64 arithmetic, the algorithms of the
reference's DAF/MAF/ATF Faster R-CNN training path so that the MI355X HIP path can be
checked against it.  Every function cites the reference file:line it follows
(paths relative to the reference checkout, ``lib/...``).

Rules (enforced by review):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
    may import this package, and only as the *checker* / CPU baseline — never as the
    thing measured or shipped.  The product path (``tlod``) never imports it and fails
    loudly if its HIP library is missing.
  * Semantics are those of the reference's CUDA kernels and torch-CUDA ops, NOT of the
    reference's buggy CPU fallbacks (``nms_cpu.py:23-24``, ``roi_align.c:175``,
    ``roi_pool.py:21-23``).
  * Float ops are IEEE single precision, each op rounded, in source order (no FMA
    contraction); where the CUDA source promotes to double (``1.`` literals in
    ``roi_align_kernel.cu``) the restatement computes in float64.

Pinning: the anchor generator is pinned by the reference's only known-answer vector
(``lib/model/rpn/generate_anchors.py:29-37``, MATLAB 1-based, Python = value - 1).
Everything else is **parity unpinned**: the reference ships no tests/fixtures for these
ops, cannot be built here (legacy THC/cffi + nvcc) and importing it was denied by the
environment.  Golden fixtures under ``tests/golden`` are generated from
this restatement by ``tests/golden/make_golden.py``.
"""
