"""Fused losses (csrc/losses.hip) vs the torch compositions that restate the reference:
RPN masked cross entropy + smooth-L1 (rpn.py:89-108, net_utils.py:72-86), the RCNN head's
cross entropy + gathered smooth-L1 (faster_rcnn.py:158-177), and the six DAF domain losses
(faster_rcnn.py:181-220, LabelResizeLayer.py:18-57).  Values and input gradients agree to
fp32 reduction-order error (rtol 2e-5 / atol 1e-7 relative to the gradient scale)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def close(a, b, rtol=2e-5):
    a, b = a.double(), b.double()
    scale = b.abs().max().item() + 1e-30
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert err <= rtol * scale + 1e-12, (err, scale)


def rpn_inputs(B, A, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    score = torch.randn(B, 2 * A, H, W, generator=g) * 3
    bbox = torch.randn(B, 4 * A, H, W, generator=g)
    lab = torch.randint(-1, 2, (B, 1, A * H, W), generator=g).float()
    lab[(torch.rand(lab.shape, generator=g) < 0.9)] = -1.0  # mostly ignored, like sampling
    tgt = torch.randn(B, 4 * A, H, W, generator=g) * 0.3
    inside = (torch.rand(B, 4 * A, H, W, generator=g) < 0.3).float()
    outside = inside * 0.01
    return [t.to(dev) for t in (score, bbox, lab, tgt, inside, outside)]


@pytest.mark.parametrize("B,A,H,W", [(1, 9, 37, 75), (2, 9, 5, 7), (1, 3, 1, 1)])
def test_rpn_loss(B, A, H, W):
    from tlod.detector.losses import masked_cross_entropy, rpn_losses, smooth_l1_loss
    from tlod.rpn.rpn_head import _RPN
    score, bbox, lab, tgt, inside, outside = rpn_inputs(B, A, H, W, B * 1000 + H)
    s1, b1 = score.clone().requires_grad_(True), bbox.clone().requires_grad_(True)
    lc, lb = rpn_losses(s1, b1, lab, tgt, inside, outside, sigma=3.0)
    (2.0 * lc + 0.5 * lb).backward()
    s2, b2 = score.clone().requires_grad_(True), bbox.clone().requires_grad_(True)
    sr = _RPN.reshape(s2, 2)
    scores = sr.permute(0, 2, 3, 1).contiguous().view(-1, 2)
    rc = masked_cross_entropy(scores, lab.view(B, -1).view(-1))
    rb = smooth_l1_loss(b2, tgt, inside, outside, sigma=3, dim=[1, 2, 3])
    (2.0 * rc + 0.5 * rb).backward()
    close(lc, rc)
    close(lb, rb)
    close(s1.grad, s2.grad)
    close(b1.grad, b2.grad)


def test_rpn_loss_all_ignored():
    from tlod.detector.losses import rpn_losses
    score, bbox, lab, tgt, inside, outside = rpn_inputs(1, 9, 4, 4, 3)
    lab.fill_(-1.0)
    s1 = score.clone().requires_grad_(True)
    lc, lb = rpn_losses(s1, bbox, lab, tgt, inside, outside)
    lc.backward()
    assert lc.item() == 0.0 and torch.count_nonzero(s1.grad).item() == 0


@pytest.mark.parametrize("R,C,agnostic", [(256, 9, False), (512, 21, False), (37, 9, True)])
def test_rcnn_loss(R, C, agnostic):
    from tlod.detector.losses import rcnn_losses, smooth_l1_loss
    g = torch.Generator().manual_seed(R + C)
    cls = (torch.randn(R, C, generator=g) * 2).to(dev)
    box = torch.randn(R, 4 if agnostic else 4 * C, generator=g).to(dev)
    lab = torch.randint(0, C, (R,), generator=g).to(dev)
    lab[: R // 4] = 0  # background rows
    tgt = (torch.randn(R, 4, generator=g) * 0.5).to(dev)
    inside = (lab > 0).float()[:, None].expand(R, 4).contiguous()
    outside = inside.clone()
    c1, b1 = cls.clone().requires_grad_(True), box.clone().requires_grad_(True)
    prob, sel, lc, lb = rcnn_losses(c1, b1, lab, tgt, inside, outside, agnostic)
    (lc + 3.0 * lb).backward()
    c2, b2 = cls.clone().requires_grad_(True), box.clone().requires_grad_(True)
    bp = b2
    if not agnostic:
        bp = torch.gather(b2.view(R, C, 4), 1, lab.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1)
    rc = F.cross_entropy(c2, lab)
    rb = smooth_l1_loss(bp, tgt, inside, outside)
    (rc + 3.0 * rb).backward()
    close(prob, F.softmax(cls, 1))
    assert torch.equal(sel, bp.detach())
    close(lc, rc)
    close(lb, rb)
    close(c1.grad, c2.grad)
    close(b1.grad, b2.grad)


def da_reference(ss, st, ins_s, ins_t, need_s, need_t):
    from tlod.da.daf import image_label, instance_label
    mse = torch.nn.MSELoss(reduction="sum")
    da_img = F.nll_loss(F.log_softmax(ss, 1), image_label(ss, need_s))
    tgt_da_img = F.nll_loss(F.log_softmax(st, 1), image_label(st, need_t))
    da_ins = F.binary_cross_entropy(ins_s, instance_label(ins_s.shape[0], need_s))
    tgt_da_ins = F.binary_cross_entropy(ins_t, instance_label(ins_t.shape[0], need_t))
    cons_s = F.softmax(ss, 1)[:, 1, :, :].mean()
    cons_t = F.softmax(st, 1)[:, 0, :, :].mean()
    da_cst = mse(ins_s, cons_s.detach().expand_as(ins_s))
    tgt_da_cst = mse(ins_t, cons_t.detach().expand_as(ins_t))
    return da_img, da_ins, tgt_da_img, tgt_da_ins, da_cst, tgt_da_cst


@pytest.mark.parametrize("Bs,Bt,Hs,Ws,Ht,Wt,n_s,n_t", [
    (1, 1, 37, 75, 37, 75, 256, 300),      # the DAF step (source 256 sampled, target 300)
    (2, 1, 9, 11, 5, 6, 512, 300),         # two source images: rows 256.. get need[1]
    (1, 1, 4, 4, 3, 5, 0, 7)])             # no source instances
def test_da_losses(Bs, Bt, Hs, Ws, Ht, Wt, n_s, n_t):
    from tlod.detector.losses import daf_da_losses
    g = torch.Generator().manual_seed(Bs * 7 + n_t)
    ss = (torch.randn(Bs, 2, Hs, Ws, generator=g) * 2).to(dev)
    st = (torch.randn(Bt, 2, Ht, Wt, generator=g) * 2).to(dev)
    ins_s = torch.rand(n_s, 1, generator=g).to(dev)
    ins_t = torch.rand(n_t, 1, generator=g).to(dev)
    if n_t > 2:
        ins_t[0, 0], ins_t[1, 0] = 1.0, 0.0  # log clamps at -100 and the 1e-12 grad floor
    need_s = torch.tensor([1.0, 0.0][:Bs], device=dev)
    need_t = torch.zeros(Bt, device=dev)
    w = torch.tensor([1.0, 0.5, 2.0, 0.25, 3.0, 0.125], device=dev)
    xs = [t.clone().requires_grad_(True) for t in (ss, st, ins_s, ins_t)]
    got = daf_da_losses(*xs, need_s, need_t)
    (torch.stack(got) @ w).backward()
    ys = [t.clone().requires_grad_(True) for t in (ss, st, ins_s, ins_t)]
    ref = da_reference(*ys, need_s, need_t)
    if n_s == 0:  # torch's BCE / nll on empty input is NaN; the fused loss reports 0
        assert got[1].item() == 0.0 and got[4].item() == 0.0
        ref = tuple(r if i not in (1, 4) else torch.zeros((), device=dev)
                    for i, r in enumerate(ref))
        (torch.stack([r for r in ref]) @ w).backward()
    else:
        (torch.stack(ref) @ w).backward()
    for a, b in zip(got, ref):
        close(a, b)
    for a, b in zip(xs, ys):
        if b.grad is None:
            assert a.grad is None or a.grad.numel() == 0 or torch.count_nonzero(a.grad) == 0
        else:
            close(a.grad, b.grad)


def test_rpn_loss_partial_batch():
    """Loss over the first image of a 2-image head batch: the gradient of the second image
    is zero and the first matches the single-image loss."""
    from tlod.detector.losses import rpn_losses
    score, bbox, lab, tgt, inside, outside = rpn_inputs(1, 12, 37, 75, 11)
    g = torch.Generator().manual_seed(12)
    score2 = torch.cat([score, torch.randn(score.shape, generator=g).to(dev)], 0)
    bbox2 = torch.cat([bbox, torch.randn(bbox.shape, generator=g).to(dev)], 0)
    s2, b2 = score2.clone().requires_grad_(True), bbox2.clone().requires_grad_(True)
    lc2, lb2 = rpn_losses(s2, b2, lab, tgt, inside, outside)
    (lc2 + lb2).backward()
    s1, b1 = score.clone().requires_grad_(True), bbox.clone().requires_grad_(True)
    lc1, lb1 = rpn_losses(s1, b1, lab, tgt, inside, outside)
    (lc1 + lb1).backward()
    assert torch.equal(lc1, lc2) and torch.equal(lb1, lb2)
    assert torch.equal(s2.grad[:1], s1.grad) and torch.equal(b2.grad[:1], b1.grad)
    assert torch.count_nonzero(s2.grad[1:]) == 0 and torch.count_nonzero(b2.grad[1:]) == 0


def test_rcnn_loss_partial_rows():
    from tlod.detector.losses import rcnn_losses
    g = torch.Generator().manual_seed(3)
    R, Rt, C = 256, 556, 9
    cls = torch.randn(Rt, C, generator=g).to(dev)
    box = torch.randn(Rt, 4 * C, generator=g).to(dev)
    lab = torch.randint(0, C, (R,), generator=g).to(dev)
    tgt = torch.randn(R, 4, generator=g).to(dev)
    w = (lab > 0).float()[:, None].expand(R, 4).contiguous()
    c2, b2 = cls.clone().requires_grad_(True), box.clone().requires_grad_(True)
    p2, s2, lc2, lb2 = rcnn_losses(c2, b2, lab, tgt, w, w)
    (lc2 + 2 * lb2).backward()
    c1, b1 = cls[:R].clone().requires_grad_(True), box[:R].clone().requires_grad_(True)
    p1, s1, lc1, lb1 = rcnn_losses(c1, b1, lab, tgt, w, w)
    (lc1 + 2 * lb1).backward()
    assert torch.equal(p1, p2) and torch.equal(s1, s2)
    assert torch.equal(lc1, lc2) and torch.equal(lb1, lb2)
    assert torch.equal(c2.grad[:R], c1.grad) and torch.equal(b2.grad[:R], b1.grad)
    assert torch.count_nonzero(c2.grad[R:]) == 0 and torch.count_nonzero(b2.grad[R:]) == 0


def test_da_losses_packed_matches_split():
    from tlod.detector.losses import daf_da_losses, daf_da_losses_packed
    g = torch.Generator().manual_seed(21)
    sc = (torch.randn(2, 2, 37, 75, generator=g) * 2).to(dev)
    ins = torch.rand(556, 1, generator=g).to(dev)
    need_s, need_t = torch.ones(1, device=dev), torch.zeros(1, device=dev)
    w = torch.tensor([1.0, 0.5, 2.0, 0.25, 3.0, 0.125], device=dev)
    a_sc, a_in = sc.clone().requires_grad_(True), ins.clone().requires_grad_(True)
    got = daf_da_losses_packed(a_sc, a_in, 1, 256, need_s, need_t)
    (torch.stack(got) @ w).backward()
    xs = [t.clone().requires_grad_(True) for t in (sc[:1], sc[1:], ins[:256], ins[256:])]
    ref = daf_da_losses(*xs, need_s, need_t)
    (torch.stack(ref) @ w).backward()
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    assert torch.equal(a_sc.grad, torch.cat([xs[0].grad, xs[1].grad], 0))
    assert torch.equal(a_in.grad, torch.cat([xs[2].grad, xs[3].grad], 0))
