"""Detector losses (lib/model/utils/net_utils.py:72-86, lib/model/rpn/rpn.py:89-108)."""
import torch
import torch.nn.functional as F

from .. import _lib


def fused_losses():
    """TLOD_FUSED_LOSSES (default 1): the one-launch libtlod losses below; 0 = the torch
    compositions (A/B comparison and tests)."""
    return _lib.env("TLOD_FUSED_LOSSES", "1") != "0"


def smooth_l1_loss(bbox_pred, bbox_targets, inside_w, outside_w, sigma=1.0, dim=(1,)):
    """_smooth_l1_loss (net_utils.py:72-86): sum over `dim` (descending), then mean."""
    sigma_2 = sigma ** 2
    in_box_diff = inside_w * (bbox_pred - bbox_targets)
    abs_d = in_box_diff.abs()
    sign = (abs_d < 1.0 / sigma_2).detach().float()
    in_loss = in_box_diff.pow(2) * (sigma_2 / 2.0) * sign + (abs_d - 0.5 / sigma_2) * (1.0 - sign)
    loss = outside_w * in_loss
    for i in sorted(dim, reverse=True):
        loss = loss.sum(i)
    return loss.mean()


def masked_cross_entropy(scores, labels, ignore=-1):
    """F.cross_entropy over the rows with label != ignore, averaged — the reference selects
    those rows with nonzero()+index_select (rpn.py:92-97, a host sync); this masks instead."""
    lab = labels.long()
    keep = (lab != ignore)
    ce = F.cross_entropy(scores, lab.clamp(min=0), reduction="none")
    return (ce * keep).sum() / keep.sum().clamp(min=1)


_WEIGHTS = {}


def weighted_loss_sum(terms, weights):
    """sum_i weights[i] * terms[i].mean() (the methods' loss sums, e.g. DAF_train.py:397-400)
    as one stack + one dot product instead of a kernel per .mean(), product and addition
    (the terms are scalars, so .mean() is the identity)."""
    t = torch.stack([x.reshape(()) if x.numel() == 1 else x.mean() for x in terms])
    key = (str(t.device), tuple(float(w) for w in weights))
    w = _WEIGHTS.get(key)
    if w is None:
        w = torch.tensor(key[1], dtype=t.dtype, device=t.device)
        _WEIGHTS[key] = w
    return torch.dot(t, w)


# ---------------------------------------------------------------------------- fused losses
# One libtlod launch per loss family forward and one per backward (csrc/losses.hip),
# replacing the ~200 small torch kernels the compositions above issue per training step.
# The compositions stay as the readable statement of the math (and the tests' reference).

def _grad_pair(*gs):
    """The upstream gradients of adjacent scalar losses as one contiguous device vector:
    weighted_loss_sum's backward already lays them out adjacently (views of one tensor),
    in which case no kernel is needed."""
    g0 = gs[0]
    if all(g is not None and g.dtype == torch.float32 and g.numel() == 1 for g in gs) and \
            all(g.data_ptr() == g0.data_ptr() + 4 * i for i, g in enumerate(gs)):
        return g0
    z = None
    out = []
    dev = next(g.device for g in gs if g is not None)
    for g in gs:
        if g is None:
            z = z if z is not None else torch.zeros((), dtype=torch.float32, device=dev)
            g = z
        out.append(g.reshape(()).float())
    return torch.stack(out)


class RPNLossFunction(torch.autograd.Function):
    """(rpn_loss_cls, rpn_loss_box) of _RPN (rpn.py:89-108) from the raw RPN_cls_score
    (B_total, 2A, H, W) and RPN_bbox_pred: tlod_rpn_loss_f32 / _bwd_f32.  The loss covers
    the first B = labels.shape[0] images (the source image of a batched source + target
    head pass); the gradients cover all B_total, so no slice enters the autograd graph."""

    @staticmethod
    def forward(ctx, score, bbox, labels, targets, inside, outside, sigma):
        from .. import _lib
        _lib.require_cuda(score, bbox, labels, targets, inside, outside)
        B_total, twoA, H, W = score.shape
        A = twoA // 2
        B = labels.shape[0]
        t = [x.detach().contiguous().float() for x in (score, bbox, labels, targets, inside,
                                                       outside)]
        assert t[1].shape == (B_total, 4 * A, H, W) and t[2].numel() == B * A * H * W
        assert B <= B_total and t[3].shape == (B, 4 * A, H, W)
        loss = torch.empty(3, dtype=torch.float32, device=score.device)  # cls, box, count
        L = _lib.lib()
        abi = [t[0], t[2], t[1], t[3], t[4], t[5]]  # score, labels, bbox, targets, in, out
        _lib.check(L.tlod_rpn_loss_f32(*[_lib.ptr(x) for x in abi], B, A, H, W, float(sigma),
                                       _lib.ptr(loss), _lib.ptr(loss[2:]), _lib.stream_of(score)),
                   "rpn_loss")
        ctx.sigma, ctx.dims = sigma, (B, B_total, A, H, W)
        ctx.save_for_backward(*t, loss)
        return loss[0], loss[1]

    @staticmethod
    def backward(ctx, g_cls, g_box):
        from .. import _lib
        *t, loss = ctx.saved_tensors
        B, B_total, A, H, W = ctx.dims
        g = _grad_pair(g_cls, g_box)
        dscore = torch.empty_like(t[0])
        dbbox = torch.empty_like(t[1])
        L = _lib.lib()
        abi = [t[0], t[2], t[1], t[3], t[4], t[5]]
        _lib.check(L.tlod_rpn_loss_bwd_f32(*[_lib.ptr(x) for x in abi], B, B_total, A, H, W,
                                           float(ctx.sigma), _lib.ptr(g), _lib.ptr(loss[2:]),
                                           _lib.ptr(dscore), _lib.ptr(dbbox),
                                           _lib.stream_of(dscore)), "rpn_loss_bwd")
        return dscore, dbbox, None, None, None, None, None


def rpn_losses(rpn_cls_score, bbox, labels, targets, inside, outside, sigma=3.0):
    """Fused masked cross entropy + smooth-L1 of the RPN; returns (loss_cls, loss_box)."""
    return RPNLossFunction.apply(rpn_cls_score, bbox, labels, targets, inside, outside, sigma)


class RCNNLossFunction(torch.autograd.Function):
    """cls_prob, gathered bbox_pred, RCNN_loss_cls, RCNN_loss_bbox of the detection head
    (faster_rcnn.py:158-177) in one launch: tlod_rcnn_loss_f32 / _bwd_f32."""

    @staticmethod
    def forward(ctx, cls_score, bbox_pred, labels, targets, inside, outside, agnostic, sigma):
        from .. import _lib
        _lib.require_cuda(cls_score, bbox_pred, labels, targets, inside, outside)
        ctx.set_materialize_grads(False)  # cls_prob / gathered boxes get no gradient
        R_total, C = cls_score.shape
        R = labels.numel()  # the loss covers the first R rows (the source RoIs)
        cs, bp = cls_score.detach().contiguous().float(), bbox_pred.detach().contiguous().float()
        lab = labels.detach().contiguous().long()
        tg, iw, ow = (x.detach().contiguous().float() for x in (targets, inside, outside))
        assert bp.shape == (R_total, 4 if agnostic else 4 * C) and R <= R_total
        assert tg.shape == iw.shape == ow.shape == (R, 4)
        prob = torch.empty((R, C), dtype=torch.float32, device=cs.device)
        sel = torch.empty((R, 4), dtype=torch.float32, device=cs.device)
        loss = torch.empty(2, dtype=torch.float32, device=cs.device)
        L = _lib.lib()
        _lib.check(L.tlod_rcnn_loss_f32(_lib.ptr(cs), _lib.ptr(bp), _lib.ptr(lab), _lib.ptr(tg),
                                        _lib.ptr(iw), _lib.ptr(ow), R, C, int(agnostic),
                                        float(sigma), _lib.ptr(prob), _lib.ptr(sel),
                                        _lib.ptr(loss), _lib.stream_of(cs)), "rcnn_loss")
        ctx.agnostic, ctx.sigma, ctx.R_total = agnostic, sigma, R_total
        ctx.save_for_backward(prob, bp, lab, tg, iw, ow)
        ctx.mark_non_differentiable(prob, sel)
        return prob, sel, loss[0], loss[1]

    @staticmethod
    def backward(ctx, g_prob, g_sel, g_cls, g_box):
        from .. import _lib
        prob, bp, lab, tg, iw, ow = ctx.saved_tensors
        R, C = prob.shape
        if g_cls is None and g_box is None:
            return None, None, None, None, None, None, None, None
        g = _grad_pair(g_cls, g_box)
        dcls = torch.empty((ctx.R_total, C), dtype=torch.float32, device=prob.device)
        dbox = torch.empty_like(bp)
        L = _lib.lib()
        _lib.check(L.tlod_rcnn_loss_bwd_f32(_lib.ptr(prob), _lib.ptr(bp), _lib.ptr(lab),
                                            _lib.ptr(tg), _lib.ptr(iw), _lib.ptr(ow), R,
                                            ctx.R_total, C,
                                            int(ctx.agnostic), float(ctx.sigma), _lib.ptr(g),
                                            _lib.ptr(dcls), _lib.ptr(dbox),
                                            _lib.stream_of(prob)), "rcnn_loss_bwd")
        return dcls, dbox, None, None, None, None, None, None


def rcnn_losses(cls_score, bbox_pred, labels, targets, inside, outside, agnostic=False,
                sigma=1.0):
    """Training-mode head losses over the first labels.numel() rows of cls_score /
    bbox_pred: returns (cls_prob, bbox_pred gathered at the label's class (a copy of
    bbox_pred when class-agnostic), loss_cls, loss_bbox) for those rows.  cls_prob and
    the gathered boxes are outputs only (no gradient flows back through them, as in
    training, where only the losses are differentiated)."""
    return RCNNLossFunction.apply(cls_score, bbox_pred, labels, targets, inside, outside,
                                  bool(agnostic), sigma)


class DALossFunction(torch.autograd.Function):
    """The six DAF domain losses (faster_rcnn.py:181-220) of the source and target
    domains in one launch: tlod_da_loss_f32 / _bwd_f32."""

    @staticmethod
    def forward(ctx, score_s, score_t, ins_s, ins_t, need_s, need_t):
        from .. import _lib
        _lib.require_cuda(score_s, score_t, ins_s, ins_t)
        t = [x.detach().contiguous().float() for x in (score_s, score_t)]
        ins = [x.detach().contiguous().float().view(-1) for x in (ins_s, ins_t)]
        need = [x.detach().to(score_s.device).contiguous().float().view(-1)
                for x in (need_s, need_t)]
        (Bs, cs, Hs, Ws), (Bt, ct, Ht, Wt) = t[0].shape, t[1].shape
        assert cs == 2 and ct == 2 and need[0].numel() == Bs and need[1].numel() == Bt
        out = torch.empty(8, dtype=torch.float32, device=score_s.device)  # 6 losses, 2 cons
        L = _lib.lib()
        _lib.check(L.tlod_da_loss_f32(_lib.ptr(t[0]), _lib.ptr(t[1]), _lib.ptr(need[0]),
                                      _lib.ptr(need[1]), _lib.ptr(ins[0]), _lib.ptr(ins[1]), Bs,
                                      Bt, Hs, Ws, Ht, Wt, ins[0].numel(), ins[1].numel(),
                                      _lib.ptr(out), _lib.ptr(out[6:]), _lib.stream_of(t[0])),
                   "da_loss")
        ctx.dims = (Bs, Bt, Hs, Ws, Ht, Wt)
        ctx.ins_shapes = (ins_s.shape, ins_t.shape)
        ctx.save_for_backward(*t, *ins, *need, out)
        # reference order: DA_img_loss_cls, DA_ins_loss_cls, tgt_DA_img_loss_cls,
        # tgt_DA_ins_loss_cls, DA_cst_loss, tgt_DA_cst_loss
        return out[0], out[1], out[3], out[4], out[2], out[5]

    @staticmethod
    def backward(ctx, g_img_s, g_ins_s, g_img_t, g_ins_t, g_cst_s, g_cst_t):
        from .. import _lib
        ss, st, ins_s, ins_t, need_s, need_t, out = ctx.saved_tensors
        Bs, Bt, Hs, Ws, Ht, Wt = ctx.dims
        g = torch.stack([x.reshape(()) if x is not None else out.new_zeros(())
                         for x in (g_img_s, g_ins_s, g_cst_s, g_img_t, g_ins_t, g_cst_t)])
        ds, dt = torch.empty_like(ss), torch.empty_like(st)
        di_s, di_t = torch.empty_like(ins_s), torch.empty_like(ins_t)
        L = _lib.lib()
        _lib.check(L.tlod_da_loss_bwd_f32(_lib.ptr(ss), _lib.ptr(st), _lib.ptr(need_s),
                                          _lib.ptr(need_t), _lib.ptr(ins_s), _lib.ptr(ins_t), Bs,
                                          Bt, Hs, Ws, Ht, Wt, ins_s.numel(), ins_t.numel(),
                                          _lib.ptr(g), _lib.ptr(out[6:]), _lib.ptr(ds),
                                          _lib.ptr(dt), _lib.ptr(di_s), _lib.ptr(di_t),
                                          _lib.stream_of(ss)), "da_loss_bwd")
        return (ds, dt, di_s.view(ctx.ins_shapes[0]), di_t.view(ctx.ins_shapes[1]), None, None)


class DALossPackedFunction(torch.autograd.Function):
    """DALossFunction with the two domains packed along the batch / row axis of one image
    score tensor (Bs + Bt, 2, H, W) and one instance tensor (n_s + n_t, 1) — the layout of
    DAF's batched source + target pass — so each gets one gradient tensor and no slice
    enters the autograd graph."""

    @staticmethod
    def forward(ctx, score2, ins2, Bs, n_s, need_s, need_t):
        from .. import _lib
        _lib.require_cuda(score2, ins2)
        sc = score2.detach().contiguous().float()
        ins = ins2.detach().contiguous().float().view(-1)
        B2, c2, H, W = sc.shape
        Bt, n_t = B2 - Bs, ins.numel() - n_s
        need = [x.detach().to(sc.device).contiguous().float().view(-1) for x in (need_s, need_t)]
        assert c2 == 2 and Bt > 0 and n_t >= 0 and need[0].numel() == Bs and need[1].numel() == Bt
        out = torch.empty(8, dtype=torch.float32, device=sc.device)
        img = 2 * H * W * 4  # bytes per image of score2
        L = _lib.lib()
        _lib.check(L.tlod_da_loss_f32(_lib.ptr(sc), _lib.c_void_p(sc.data_ptr() + Bs * img),
                                      _lib.ptr(need[0]), _lib.ptr(need[1]), _lib.ptr(ins),
                                      _lib.c_void_p(ins.data_ptr() + 4 * n_s), Bs, Bt, H, W, H,
                                      W, n_s, n_t, _lib.ptr(out), _lib.ptr(out[6:]),
                                      _lib.stream_of(sc)), "da_loss")
        ctx.dims = (Bs, Bt, H, W, n_s, n_t)
        ctx.ins_shape = ins2.shape
        ctx.save_for_backward(sc, ins, need[0], need[1], out)
        return out[0], out[1], out[3], out[4], out[2], out[5]

    @staticmethod
    def backward(ctx, g_img_s, g_ins_s, g_img_t, g_ins_t, g_cst_s, g_cst_t):
        from .. import _lib
        sc, ins, need_s, need_t, out = ctx.saved_tensors
        Bs, Bt, H, W, n_s, n_t = ctx.dims
        g = torch.stack([x.reshape(()) if x is not None else out.new_zeros(())
                         for x in (g_img_s, g_ins_s, g_cst_s, g_img_t, g_ins_t, g_cst_t)])
        dsc, dins = torch.empty_like(sc), torch.empty_like(ins)
        img = 2 * H * W * 4
        L = _lib.lib()
        _lib.check(L.tlod_da_loss_bwd_f32(
            _lib.ptr(sc), _lib.c_void_p(sc.data_ptr() + Bs * img), _lib.ptr(need_s),
            _lib.ptr(need_t), _lib.ptr(ins), _lib.c_void_p(ins.data_ptr() + 4 * n_s), Bs, Bt, H,
            W, H, W, n_s, n_t, _lib.ptr(g), _lib.ptr(out[6:]), _lib.ptr(dsc),
            _lib.c_void_p(dsc.data_ptr() + Bs * img), _lib.ptr(dins),
            _lib.c_void_p(dins.data_ptr() + 4 * n_s), _lib.stream_of(sc)), "da_loss_bwd")
        return dsc, dins.view(ctx.ins_shape), None, None, None, None


def daf_da_losses_packed(score2, ins2, Bs, n_s, need_s, need_t):
    """daf_da_losses for the packed (source rows first) layout of DALossPackedFunction."""
    return DALossPackedFunction.apply(score2, ins2, int(Bs), int(n_s), need_s, need_t)


def daf_da_losses(base_score_s, base_score_t, ins_s, ins_t, need_s, need_t):
    """(DA_img, DA_ins, tgt_DA_img, tgt_DA_ins, DA_cst, tgt_DA_cst) of DAF in two launches
    (forward + backward)."""
    return DALossFunction.apply(base_score_s, base_score_t, ins_s, ins_t, need_s, need_t)
