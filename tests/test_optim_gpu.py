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


def test_fast_table_key_matches_slow_path(monkeypatch):
    """The descriptor table's fast key (every gradient arrived in its arena slot since the
    last zero_grad: no per-parameter host work) against the optimizer without an arena
    (per-pointer key every step), over steps with all gradients, a step where one module
    gets none, and a step with no zero_grad in between: parameters bit-identical."""
    from tlod.optim import FusedSGDClip

    def build(arena):
        monkeypatch.setenv("TLOD_GRAD_ARENA", "1" if arena else "0")
        torch.manual_seed(0)
        m1, m2 = torch.nn.Linear(64, 32).cuda(), torch.nn.Linear(32, 16).cuda()
        opt = FusedSGDClip([{"params": list(m1.parameters()) + list(m2.parameters()),
                             "lr": 0.05, "weight_decay": 5e-4}], clip_norm=1.0)
        return m1, m2, opt
    runs = []
    for arena in (True, False):
        m1, m2, opt = build(arena)
        g = torch.Generator(device="cuda").manual_seed(1)
        for step, (both, zero) in enumerate([(1, 1), (1, 1), (0, 1), (1, 1), (1, 0), (1, 1)]):
            if zero:
                opt.zero_grad()
            x = torch.randn(8, 64, device="cuda", generator=g)
            h = m1(x)
            (m2(h).square().mean() if both else h.square().mean()).backward()
            opt.step()
        if arena:
            assert opt.table_builds <= 3  # all-gradient steps share one table
        runs.append([p.detach().clone() for p in list(m1.parameters()) + list(m2.parameters())])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("clip", [0.0, 10.0])
def test_fused_pack_update(clip, monkeypatch):
    """tlod_sgd_clip_pack_f32: the 3x3 weights a FusedSGDClip owns are updated by tiles that
    also write their split-bf16 packs.  After every step the packs the convs will use (the
    cached ones: no re-pack, PACK_GEN unchanged) are bit-identical to packs made from the
    updated weights, and the weights match the chunk-only update (TLOD_SGD_PACK=0) bit for
    bit, with and without clipping (the norm's chunk rows are in parameter order either way,
    round-5 advisor).  Ragged
    channel counts (tiles past the last channel), a BN-scaled input-gradient pack, Cin = 3."""
    from tlod import conv
    from tlod.optim import FusedSGDClip
    shapes = [(40, 24), (64, 64), (80, 36), (256, 128), (16, 3), (33, 65)]
    g = torch.Generator(device="cuda").manual_seed(1)

    def params():
        torch.manual_seed(3)
        ws = [torch.nn.Parameter(torch.randn(co, ci, 3, 3, device="cuda") * 0.05) for co, ci in shapes]
        return ws + [torch.nn.Parameter(torch.randn(40, device="cuda"))]

    pa, pb = params(), params()
    scale = torch.rand(80, device="cuda") + 0.5
    groups = lambda ps: [{"params": ps[:-1], "lr": 0.01, "weight_decay": 5e-4},
                         {"params": ps[-1:], "lr": 0.02, "weight_decay": 0.0}]
    monkeypatch.setenv("TLOD_SGD_PACK", "1")
    fo = FusedSGDClip(groups(pa), momentum=0.9, clip_norm=clip)
    monkeypatch.setenv("TLOD_SGD_PACK", "0")
    ro = FusedSGDClip(groups(pb), momentum=0.9, clip_norm=clip)
    assert all(getattr(w, "_tlod_pack_owner", False) for w in pa[:-1])
    assert not any(getattr(w, "_tlod_pack_owner", False) for w in pb)

    def packs():
        out = []
        for w in pa[:-1]:
            out += [conv.pack_bs(w, False), conv.pack_bs(w, True)]
        return out + [conv.pack_bs(pa[2], True, scale)]
    first = packs()
    gen = conv.PACK_GEN[0]
    for step in range(3):
        rs = [torch.randn(p.shape, device="cuda", generator=g) for p in pa]
        for ps, opt in ((pa, fo), (pb, ro)):
            opt.zero_grad()
            sum((p * r).sum() for p, r in zip(ps, rs)).backward()
            opt.step()
        for a, b in zip(pa, pb):
            assert torch.equal(a.detach(), b.detach())
        now = packs()
        assert conv.PACK_GEN[0] == gen and all(x is y for x, y in zip(now, first))
        fresh = []
        for w in pa[:-1]:
            fresh += [conv._pack_bs(w, False), conv._pack_bs(w, True)]
        fresh.append(conv._pack_bs(pa[2], True, scale))
        for i, (x, y) in enumerate(zip(now, fresh)):
            assert torch.equal(x, y), (step, i)
    # a trainable weight no fused optimizer owns is packed afresh on every use
    w = torch.nn.Parameter(torch.randn(8, 8, 3, 3, device="cuda"))
    assert conv.pack_bs(w, False) is not conv.pack_bs(w, False)


@pytest.mark.parametrize("order", ["plain_after", "plain_before"])
def test_plain_update_never_leaves_stale_packs(order, monkeypatch):
    """Round-5 advisor: a weight owned by a pack-writing FusedSGDClip that another optimizer
    updates with the plain kernel (TLOD_SGD_PACK=0; its writes bump no version).  Built after
    the owner, the plain optimizer takes the ownership back; built before, it drops the
    owner's cached packs after each of its steps.  Either way the pack the next conv gets is
    bit-identical to a fresh pack of the current weight."""
    from tlod import conv
    from tlod.optim import FusedSGDClip
    torch.manual_seed(5)
    w = torch.nn.Parameter(torch.randn(48, 40, 3, 3, device="cuda") * 0.05)
    mk = lambda packs: (monkeypatch.setenv("TLOD_SGD_PACK", "1" if packs else "0"),
                        FusedSGDClip([{"params": [w], "lr": 0.01, "weight_decay": 5e-4}],
                                     momentum=0.9, clip_norm=10.0))[1]
    if order == "plain_after":
        fused, plain = mk(True), mk(False)
    else:
        plain, fused = mk(False), mk(True)
    g = torch.Generator(device="cuda").manual_seed(2)
    for opt in (fused, plain, plain, fused, plain):
        conv.pack_bs(w, False), conv.pack_bs(w, True)  # cache (or not) the current packs
        opt.zero_grad()
        (w * torch.randn(w.shape, device="cuda", generator=g)).sum().backward()
        opt.step()
        assert torch.equal(conv.pack_bs(w, False), conv._pack_bs(w, False))
        assert torch.equal(conv.pack_bs(w, True), conv._pack_bs(w, True))
