"""CPU-side checks of the C ABI boundary: the library loads, exports every symbol that
include/tlod.h declares, and the ctypes signature table covers exactly those symbols.
No compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tlod.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tlod_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("tlod_nms_f32", "tlod_roi_align_avg_fwd_f32", "tlod_proposal_f32",
                 "tlod_anchor_target_f32", "tlod_proposal_target_f32"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from tlod import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libtlod.so first (__graft_entry__.build())"
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, f"declared but not exported: {missing}"


def test_ctypes_table_matches_header():
    from tlod import _lib
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_host_only_calls():
    from tlod import _lib
    L = _lib.lib()
    assert L.tlod_abi_version() == 1
    assert L.tlod_nms_workspace_bytes(12000) >= 12000 * 188 * 8
    assert L.tlod_proposal_workspace_bytes(1, 12, 37, 75, 12000) > 0
    assert L.tlod_anchor_target_workspace_bytes(1, 12, 37, 75, 50) > 0


def test_product_path_refuses_cpu_tensors():
    import torch
    from tlod.nms import nms
    d = torch.zeros(4, 5)
    with pytest.raises((RuntimeError, NotImplementedError)):
        nms(d, 0.7)
    with pytest.raises(NotImplementedError):
        nms(d, 0.7, force_cpu=True)


def test_nhwc3_gemm_argument_checks_host_only():
    """tlod_gemm_nhwc3_bs_f32 (round 6) rejects a bad mode, channel counts whose chunks /
    column tiles would straddle taps, an epilogue on the weight gradient and an aliased
    residual — before any device work (no GPU here)."""
    import ctypes
    from tlod import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p).value
    q = p + 16

    def call(mode, C, O, residual=None, bias=None, relu=0, c=None):
        return L.tlod_gemm_nhwc3_bs_f32(mode, p, p, bias, residual, None, relu,
                                        q if c is None else c, 2, 4, 4, C, O, 6, None, 0, None)
    assert call(3, 512, 512) != 0
    assert b"mode" in L.tlod_last_error()
    assert call(0, 24, 512) != 0        # forward: C % 16
    assert call(1, 512, 40) != 0        # input gradient: O % 16
    assert call(2, 128, 512) != 0       # weight gradient: C % 256
    assert call(2, 512, 512, bias=p) != 0
    assert b"epilogue" in L.tlod_last_error()
    assert call(0, 512, 512, residual=q) != 0
    assert b"alias" in L.tlod_last_error()
