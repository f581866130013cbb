"""Detector losses (lib/model/utils/net_utils.py:72-86, lib/model/rpn/rpn.py:89-108)."""
import torch
import torch.nn.functional as F


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
