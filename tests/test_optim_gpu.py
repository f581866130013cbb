"""Fused clip_gradient + SGD (tlod_sgd_clip_f32) vs torch: clip_gradient restated from
lib/model/utils/net_utils.py:38-49 then torch.optim.SGD with the reference param groups."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("clip", [10.0, 1e-3, 0.0])
def test_fused_sgd_matches_torch(clip):
    from tlod.optim import FusedSGDClip
    torch.manual_seed(0)
    def model():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.ReLU(),
                                   torch.nn.Linear(200, 70000 // 200)).cuda()
    a, b = model(), model()

    def groups(m, lr):
        w = [p for n, p in m.named_parameters() if "bias" not in n]
        bi = [p for n, p in m.named_parameters() if "bias" in n]
        return [{"params": w, "lr": lr, "weight_decay": 5e-4},
                {"params": bi, "lr": 2 * lr, "weight_decay": 0.0}]
    fo = FusedSGDClip(groups(a, 0.01), momentum=0.9, clip_norm=clip)
    to = torch.optim.SGD(groups(b, 0.01), lr=0.01, momentum=0.9)
    for step in range(3):
        x = torch.randn(64, 300, device="cuda")
        for m, opt in ((a, fo), (b, to)):
            opt.zero_grad()
            (m(x) ** 2).mean().backward()
        fo.step()
        if clip > 0:  # clip_gradient(model, clip)
            tot = torch.sqrt(sum(p.grad.norm() ** 2 for p in b.parameters()))
            s = clip / max(float(tot), clip)
            for p in b.parameters():
                p.grad.mul_(s)
        to.step()
        for pa, pb in zip(a.parameters(), b.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)


def test_params_without_grad_are_skipped():
    """torch SGD leaves a parameter whose .grad is None untouched (no weight decay); ATF
    owns one such module (RCNN_rpn_t, lib/ATF/faster_rcnn.py:95, never called)."""
    from tlod.optim import FusedSGDClip
    torch.manual_seed(0)
    used, unused = torch.nn.Linear(8, 8).cuda(), torch.nn.Linear(8, 8).cuda()
    before = [p.detach().clone() for p in unused.parameters()]
    params = list(used.parameters()) + list(unused.parameters())
    opt = FusedSGDClip([{"params": params, "lr": 0.1, "weight_decay": 5e-4}], clip_norm=10.0)
    for _ in range(2):
        opt.zero_grad()
        used(torch.randn(4, 8, device="cuda")).sum().backward()
        opt.step()
    for p, b in zip(unused.parameters(), before):
        assert torch.equal(p.detach(), b)
    assert all(p.grad is None for p in unused.parameters())
