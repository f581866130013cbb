"""The early RPN backward (tlod/da/daf.py::early_rpn_backward, round 6): the RPN losses'
gradient computed first through a detached copy of the base feature, then joined to the
feature's gradient by a hook in the main backward, against one backward of the whole loss —
the DAF form (the head on the batched feature) and the ATF form (the head on a concatenation
of three feature rows owned by two tensors).  CPU, float64 so the comparison is exact up to
the order of a two-term sum."""
import torch

from tlod.da.daf import early_rpn_backward


def _setup(seed):
    g = torch.Generator().manual_seed(seed)
    w_base = torch.randn(6, 5, generator=g, dtype=torch.float64, requires_grad=True)
    w_t = torch.randn(6, 5, generator=g, dtype=torch.float64, requires_grad=True)
    w_rpn = torch.randn(4, 6, generator=g, dtype=torch.float64, requires_grad=True)
    w_head = torch.randn(3, 6, generator=g, dtype=torch.float64, requires_grad=True)
    x = torch.randn(2, 7, 5, generator=g, dtype=torch.float64)
    return [w_base, w_t, w_rpn, w_head], x


def _rpn_losses(w_rpn, feat):
    s = torch.tanh(feat @ w_rpn.t())
    return s.square().mean(), (s[..., :2] - 0.3).abs().sum()


def _grads(params):
    out = [None if p.grad is None else p.grad.clone() for p in params]
    for p in params:
        p.grad = None
    return out


def test_daf_form_matches_one_backward():
    params, x = _setup(0)
    w_base, _, w_rpn, w_head = params
    for early in (False, True):
        base = torch.relu(x @ w_base.t())
        rpn_in = base.detach().requires_grad_(True) if early else base
        l_cls, l_box = _rpn_losses(w_rpn, rpn_in)
        if early:
            l_cls, l_box = early_rpn_backward(l_cls, l_box, rpn_in, [(base, lambda g: g)])
            assert not l_cls.requires_grad and not l_box.requires_grad
        other = (base @ w_head.t()).sin().sum()
        (l_cls + l_box + other).backward()
        got = _grads(params)
        if early:
            for a, b in zip(ref, got):
                assert (a is None) == (b is None)
                if a is not None:
                    torch.testing.assert_close(a, b, rtol=1e-15, atol=1e-15)
        else:
            ref = got


def test_atf_form_rows_shared_by_two_features():
    """rows (source of RCNN_base, source of RCNN_base_t, target of RCNN_base) as in
    tlod/da/atf.py: the shares route rows 0 and 2 to one feature, row 1 to the other."""
    params, x = _setup(1)
    w_base, w_t, w_rpn, w_head = params
    for early in (False, True):
        bs = torch.relu(x @ w_base.t())          # (2, 7, 6): source, target
        bt = torch.relu(x[:1] @ w_t.t())         # (1, 7, 6): source through the second branch
        rpn_in = torch.cat([bs[:1], bt, bs[1:]], 0)
        if early:
            rpn_in = rpn_in.detach().requires_grad_(True)
        l_cls, l_box = _rpn_losses(w_rpn, rpn_in)
        if early:
            l_cls, l_box = early_rpn_backward(
                l_cls, l_box, rpn_in,
                [(bs, lambda g: torch.cat([g[0:1], g[2:3]], 0)), (bt, lambda g: g[1:2])])
        other = (torch.cat([bs, bt], 0) @ w_head.t()).cos().sum()
        (l_cls + l_box + other).backward()
        got = _grads(params)
        if early:
            for a, b in zip(ref, got):
                torch.testing.assert_close(a, b, rtol=1e-15, atol=1e-15)
        else:
            ref = got
