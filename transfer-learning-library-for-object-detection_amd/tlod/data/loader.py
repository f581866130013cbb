"""The training / test data layer: ``roibatchLoader`` and the batch ``sampler``
(lib/roi_data_layer/roibatchLoader.py:22-229, lib/roi_data_layer/minibatch.py:19-82,
lib/DAF/roibatchLoader.py + lib/DAF/minibatch.py:34-38 for ``need_backprop``,
methods/faster_rcnn/faster_rcnn_train.py:117-146 for the sampler).

Per item the host does what is inherently scalar — JPEG decode (PIL; the reference uses
scipy imread), the numpy RNG draws in the reference's order (scale index, gt shuffle, crop
offset), the aspect-group crop / pad geometry and the gt-box bookkeeping — and the device
builds the image blob (tlod.data.blob: BGR, flip, mean, bilinear resize, crop, zero pad,
CHW in one kernel), so the float image never exists on the host.  Items are returned as
device tensors shaped like the reference's:
    training: (data (3, Hp, Wp), im_info (3,), gt_boxes (MAX_NUM_GT_BOXES, 5),
               num_boxes () int64[, need_backprop (1,)])
    test:     (data (3, Hr, Wr), im_info (3,), gt_boxes (1, 5) = [1,1,1,1,1], num_boxes = 0
               [, need_backprop = 0])
"""
import numpy as np
import numpy.random as npr
import torch
from PIL import Image

from ..config import cfg
from .blob import image_blob, resized_size


def load_image_rgb(path):
    """scipy.misc.imread (minibatch.py:67-71): H x W x 3 uint8, grey images replicated."""
    im = Image.open(path)
    if im.mode not in ("RGB", "L"):
        im = im.convert("RGB")
    a = np.asarray(im)
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    return np.ascontiguousarray(a)


def _gt_boxes(entry, im_scale):
    """minibatch.py:39-49 (USE_ALL_GT): boxes of the fg classes, scaled, with class."""
    if cfg.TRAIN.USE_ALL_GT:
        gt_inds = np.where(entry["gt_classes"] != 0)[0]
    else:
        gt_inds = np.where((entry["gt_classes"] != 0)
                           & np.all(np.asarray(entry["gt_overlaps"]) > -1.0, axis=1))[0]
    gt = np.empty((len(gt_inds), 5), dtype=np.float32)
    gt[:, 0:4] = entry["boxes"][gt_inds, :] * im_scale
    gt[:, 4] = entry["gt_classes"][gt_inds]
    return gt


def _axis_crop(lo_box, hi_box, data_len, trim_size):
    """roibatchLoader.py:100-121 / :133-154: start of the kept window along one axis."""
    trim_size = min(trim_size, data_len)
    box_region = hi_box - lo_box + 1
    if lo_box == 0:
        return 0, trim_size
    if box_region - trim_size < 0:
        s_min = max(hi_box - trim_size, 0)
        s_max = min(lo_box, data_len - trim_size)
        s = s_min if s_min == s_max else int(np.random.choice(range(s_min, s_max)))
    else:
        add = int((box_region - trim_size) / 2)
        s = lo_box if add == 0 else int(np.random.choice(range(lo_box, lo_box + add)))
    return s, trim_size


def crop_pad_geometry(gt_boxes, data_h, data_w, ratio, need_crop):
    """roibatchLoader.py:88-200 on the host: returns (y0, x0, Hd, Wd, Ho, Wo, gt, im_hw)
    — the kept region of the resized image, the padded output size, the shifted / clamped
    gt boxes and the im_info height / width.  ``ratio`` is the group's target ratio as the
    reference stores it (a float32 tensor element: all products / quotients below are
    float32)."""
    r = np.float32(ratio)
    gt = gt_boxes.copy()
    y0 = x0 = 0
    Hd, Wd = data_h, data_w
    if need_crop:
        if r < 1:
            min_y, max_y = int(gt[:, 1].min()), int(gt[:, 3].max())
            trim = int(np.floor(np.float32(data_w) / r))
            y0, Hd = _axis_crop(min_y, max_y, data_h, trim)
            gt[:, 1] -= np.float32(y0)
            gt[:, 3] -= np.float32(y0)
            np.clip(gt[:, 1], 0, Hd - 1, out=gt[:, 1])
            np.clip(gt[:, 3], 0, Hd - 1, out=gt[:, 3])
        else:
            min_x, max_x = int(gt[:, 0].min()), int(gt[:, 2].max())
            trim = int(np.ceil(np.float32(data_h) * r))
            x0, Wd = _axis_crop(min_x, max_x, data_w, trim)
            gt[:, 0] -= np.float32(x0)
            gt[:, 2] -= np.float32(x0)
            np.clip(gt[:, 0], 0, Wd - 1, out=gt[:, 0])
            np.clip(gt[:, 2], 0, Wd - 1, out=gt[:, 2])
    if r < 1:
        Ho, Wo = int(np.ceil(np.float32(data_w) / r)), data_w
        if min(data_h, Ho) != Hd or Wd != Wo:
            raise ValueError("padding_data[:data_height] = data[0]: shape mismatch "
                             "(the reference raises here too)")
        im_hw = (Ho, data_w)
    elif r > 1:
        Ho, Wo = data_h, int(np.ceil(np.float32(data_h) * r))
        if min(data_w, Wo) != Wd or Hd != Ho:
            raise ValueError("padding_data[:, :data_width] = data[0]: shape mismatch "
                             "(the reference raises here too)")
        im_hw = (data_h, Wo)
    else:
        trim = min(data_h, data_w)
        Ho = Wo = trim
        Hd, Wd = min(Hd, trim), min(Wd, trim)
        np.clip(gt[:, :4], 0, trim, out=gt[:, :4])
        im_hw = (trim, trim)
    return y0, x0, Hd, Wd, Ho, Wo, gt, im_hw


class roibatchLoader(torch.utils.data.Dataset):
    """roibatchLoader(roidb, ratio_list, ratio_index, batch_size, num_classes, training)
    with the DAF variant's ``need_backprop`` output when ``with_need_backprop``."""

    def __init__(self, roidb, ratio_list, ratio_index, batch_size, num_classes, training=True,
                 normalize=None, device=None, with_need_backprop=False):
        self._roidb = roidb
        self._num_classes = num_classes
        self.max_num_box = cfg.MAX_NUM_GT_BOXES
        self.training = training
        self.ratio_list = ratio_list
        self.ratio_index = ratio_index
        self.batch_size = batch_size
        self.data_size = len(ratio_list)
        self.with_need_backprop = with_need_backprop
        self._device = None if device is None else torch.device(device)
        # roibatchLoader.py:36-55: one target ratio per batch (a float32 torch.Tensor there)
        self.ratio_list_batch = np.zeros(self.data_size, dtype=np.float32)
        num_batch = int(np.ceil(len(ratio_index) / batch_size))
        for i in range(num_batch):
            left = i * batch_size
            right = min((i + 1) * batch_size - 1, self.data_size - 1)
            if ratio_list[right] < 1:
                target = ratio_list[left]
            elif ratio_list[left] > 1:
                target = ratio_list[right]
            else:
                target = 1
            self.ratio_list_batch[left:right + 1] = target

    def __len__(self):
        return len(self._roidb)

    @property
    def device(self):
        if self._device is None:
            self._device = torch.device("cuda", torch.cuda.current_device())
        return self._device

    def _to_dev(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(self.device,
                                                                          non_blocking=True)

    def plan(self, index):
        """The host half of __getitem__: decode, the numpy draws in the reference's order,
        crop / pad geometry and gt bookkeeping (no device work).  Returns a dict."""
        index_ratio = int(self.ratio_index[index]) if self.training else index
        entry = self._roidb[index_ratio]
        # get_minibatch (minibatch.py:19-57)
        scale_ind = npr.randint(0, high=len(cfg.TRAIN.SCALES), size=1)
        target_size = cfg.TRAIN.SCALES[scale_ind[0]]
        img = load_image_rgb(entry["image"])
        H, W = img.shape[:2]
        im_scale = float(target_size) / float(min(H, W))  # blob.py:41-43 (MAX_SIZE unused)
        Hr, Wr = resized_size(H, im_scale), resized_size(W, im_scale)
        gt = _gt_boxes(entry, im_scale)
        need = 0.0 if entry["image"].find("source_") == -1 else 1.0
        p = dict(img=img, im_scale=im_scale, flip=bool(entry.get("flipped", False)),
                 need_backprop=need)
        if not self.training:
            p.update(crop=(0, 0), keep=(Hr, Wr), out=(Hr, Wr),
                     im_info=np.array([Hr, Wr, im_scale], np.float32),
                     gt_boxes=np.ones(5, np.float32), num_boxes=0, need_backprop=0.0)
            return p
        np.random.shuffle(gt)
        y0, x0, Hd, Wd, Ho, Wo, gt, im_hw = crop_pad_geometry(
            gt, Hr, Wr, self.ratio_list_batch[index], entry["need_crop"])
        keep = np.where(~((gt[:, 0] == gt[:, 2]) | (gt[:, 1] == gt[:, 3])))[0]
        pad = np.zeros((self.max_num_box, gt.shape[1]), np.float32)
        num_boxes = 0
        if keep.size:
            gt = gt[keep]
            num_boxes = min(gt.shape[0], self.max_num_box)
            pad[:num_boxes, :] = gt[:num_boxes]
        p.update(crop=(y0, x0), keep=(Hd, Wd), out=(Ho, Wo),
                 im_info=np.array([im_hw[0], im_hw[1], im_scale], np.float32), gt_boxes=pad,
                 num_boxes=num_boxes)
        return p

    def __getitem__(self, index):
        p = self.plan(index)
        data, _ = image_blob(self._to_dev(p["img"]), p["im_scale"], cfg.PIXEL_MEANS, p["flip"],
                             crop=p["crop"], keep_hw=p["keep"], out_hw=p["out"])
        out = (data, self._to_dev(p["im_info"]), self._to_dev(p["gt_boxes"]),
               torch.tensor(p["num_boxes"], dtype=torch.int64).to(self.device,
                                                                   non_blocking=True))
        if self.with_need_backprop:
            out += (self._to_dev(np.array([p["need_backprop"]], np.float32)),)
        return out


class sampler(torch.utils.data.Sampler):
    """faster_rcnn_train.py:117-146: a random permutation of whole batches (consecutive
    ratio-sorted indices stay together), the leftover tail appended; ``rank`` / ``world``
    stride the sequence for one-process-per-GPU data parallelism."""

    def __init__(self, train_size, batch_size, rank=0, world=1, generator=None):
        self.num_data = train_size
        self.num_per_batch = int(train_size / batch_size)
        self.batch_size = batch_size
        self.range = torch.arange(0, batch_size).view(1, batch_size).long()
        self.leftover_flag = bool(train_size % batch_size)
        if self.leftover_flag:
            self.leftover = torch.arange(self.num_per_batch * batch_size, train_size).long()
        self.rank, self.world, self.generator = rank, world, generator

    def __iter__(self):
        rand_num = torch.randperm(self.num_per_batch, generator=self.generator).view(-1, 1) \
            * self.batch_size
        view = (rand_num.expand(self.num_per_batch, self.batch_size) + self.range).view(-1)
        if self.leftover_flag:
            view = torch.cat((view, self.leftover), 0)
        return iter(view[self.rank::self.world].tolist())

    def __len__(self):
        return len(range(self.rank, self.num_data, self.world))


def collate(items):
    """Stack a batch of items (the aspect grouping gives every item of a batch one shape)."""
    return tuple(torch.stack([it[k] for it in items]) for k in range(len(items[0])))
