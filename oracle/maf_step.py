"""Oracle: the MAF VGG16 training step on the CPU (test infrastructure only).

A restatement of lib/MAF/{drm,DA,faster_rcnn}.py + methods/MAF/MAF_train.py:414-418 on
top of the DAF oracle's detector (oracle/daf_step.py: backbone, RPN, targets, RoIAlign,
heads are shared between the two methods).  The DRM is restated literally — chunk rows,
chunk columns, reshape every (B, C, s, s) chunk to (B, C*s*s, 1, 1), cat (drm.py:23-40)
— so it independently checks the device space-to-depth's channel order.  Conv/linear
arithmetic is torch-CPU fp32 ("parity unpinned" at that boundary, as for DAF).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .daf_step import OracleDAF, _GRL, forced_relu


def drm_chunks(x, scale):
    """lib/MAF/drm.py:23-40, after conv_low_dim + ReLU."""
    h_num = int(x.size(2) / scale)
    w_num = int(x.size(3) / scale)
    x = x[:, :, :int(scale * h_num), :int(scale * w_num)]
    rows = list(torch.chunk(x, h_num, dim=2))
    for i in range(len(rows)):
        rows[i] = list(torch.chunk(rows[i], w_num, dim=3))
        for j in range(len(rows[i])):
            c = rows[i][j]
            rows[i][j] = c.reshape(c.size(0), c.size(1) * scale * scale, 1, 1)
        rows[i] = torch.cat(rows[i], dim=3)
    return torch.cat(rows, dim=2)


class _WGRL(torch.autograd.Function):
    """lib/MAF/DA.py:34-53: identity; backward -alpha * score[:, dc_label] * g."""

    @staticmethod
    def forward(ctx, x, score, dc_label, alpha):
        ctx.save_for_backward(score)
        ctx.dc_label, ctx.alpha = int(dc_label), alpha
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        (score,) = ctx.saved_tensors
        w = score[:, ctx.dc_label].view(g.shape[0], 1).repeat(1, g.shape[1])
        return g.neg() * w * ctx.alpha, None, None, None


class OracleMAF(OracleDAF):
    def __init__(self, n_classes=9, dropout=0.5, backbone="vgg16"):
        super().__init__(n_classes, dropout, backbone)
        dfeat = self.RCNN_cls_score.in_features
        del self.RCNN_instanceDA
        for name, dim, inner, scale in (("RCNN_imageDA_3", 256, 64, 4), ("RCNN_imageDA_4", 512, 256, 2)):
            m = nn.Module()
            m.DRM = nn.Module()
            m.DRM.conv_low_dim = nn.Conv2d(dim, inner, 1, bias=False)
            m.Conv1 = nn.Conv2d(inner * scale * scale, 512, 1, bias=False)
            m.Conv2 = nn.Conv2d(512, 2, 1, bias=False)
            m.scale = scale
            setattr(self, name, m)
        ins = nn.Module()
        ins.dc_ip1 = nn.Linear(dfeat + n_classes, 1024)
        ins.dc_ip2 = nn.Linear(1024, 1024)
        ins.clssifer = nn.Linear(1024, 2)
        self.RCNN_instanceDA = ins

    def _image_da_drm(self, m, feat, lvl):
        """_ImageDA_drm.forward (DA.py:141-149); activation sites drm{lvl} / ida{lvl}."""
        x = _GRL.apply(feat, 0.1)
        x = drm_chunks(forced_relu(self.forced, f"drm{lvl}", m.DRM.conv_low_dim(x)), m.scale)
        return m.Conv2(forced_relu(self.forced, f"ida{lvl}", m.Conv1(x)))

    def _instance_da_w(self, x, dc_label):
        """_InstanceDA_w.forward (DA.py:90-104), no dropout.  The detached weighting pass
        feeds no gradient: plain ReLUs; the reversed pass has the sites ip1 / ip2."""
        m = self.RCNN_instanceDA

        def mlp(v, relu1, relu2):
            return m.clssifer(relu2(m.dc_ip2(relu1(m.dc_ip1(v)))))
        score = F.softmax(mlp(x.detach().clone(), F.relu, F.relu), dim=1)
        return mlp(_WGRL.apply(x, score.detach(), dc_label, 0.2),
                   lambda v: forced_relu(self.forced, "ip1", v),
                   lambda v: forced_relu(self.forced, "ip2", v))

    @staticmethod
    def _img_nll(score, label):
        lab = torch.full((score.shape[0], *score.shape[2:]), label, dtype=torch.long,
                         device=score.device)
        return F.nll_loss(F.log_softmax(score, 1), lab)

    def forward(self, batch, rng, rois_override=None):
        d = self._detect(batch, rng, rois_override)
        out = {k: d[k] for k in ("rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox",
                                 "rois")}
        for pre, lab in (("", 1), ("t_", 0)):
            s3 = self._image_da_drm(self.RCNN_imageDA_3, d[pre + "c3"], 3)
            s4 = self._image_da_drm(self.RCNN_imageDA_4, d[pre + "c4"], 4)
            s5 = self._image_da(d[pre + "base"])
            img = self._img_nll(s3, lab) + self._img_nll(s4, lab) + self._img_nll(s5, lab)
            fc7 = d[pre + "fc7"]
            cls_prob = F.softmax(self.RCNN_cls_score(fc7), 1)
            logits = self._instance_da_w(torch.cat((fc7, cls_prob), 1), lab)
            y = torch.zeros(logits.shape[0], dtype=torch.long, device=logits.device)
            y[:256] = lab  # MAF InstanceLabelResizeLayer (lib/MAF/LabelResizeLayer.py:50-60)
            ins = F.cross_entropy(logits, y)
            key = "" if lab == 1 else "tgt_"
            out[key + "DA_img_loss_cls"] = img
            out[key + "DA_ins_loss_cls"] = ins
        return out


def total_loss(o, lamda=0.1, alpha=1.0):
    """methods/MAF/MAF_train.py:415-418."""
    return (o["rpn_loss_cls"] + o["rpn_loss_box"] + o["RCNN_loss_cls"] + o["RCNN_loss_bbox"]
            + lamda * (o["DA_img_loss_cls"] + alpha * o["DA_ins_loss_cls"]
                       + o["tgt_DA_img_loss_cls"] + alpha * o["tgt_DA_ins_loss_cls"]))
