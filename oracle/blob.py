"""Oracle: the reference's data layer for one item on the CPU (TEST INFRASTRUCTURE ONLY).

Restates lib/roi_data_layer/minibatch.py:19-82 (get_minibatch / _get_image_blob),
lib/model/utils/blob.py:20-52 (im_list_to_blob / prep_im_for_blob) and
lib/roi_data_layer/roibatchLoader.py:58-229 (crop / pad / gt bookkeeping; the DAF copy
adds need_backprop, lib/DAF/minibatch.py:34-38) with numpy / torch-CPU, in the reference's
statement order and RNG call order.

cv2 is not installed, so ``cv2.resize(im, None, None, fx=s, fy=s, INTER_LINEAR)`` is
restated from OpenCV's published float path (imgproc/resize.cpp: resize() coefficient
setup, HResizeLinear, VResizeLinear): per destination column ``fx = (float)((dx + 0.5) *
(1/s) - 0.5)``, ``sx = floor(fx)``, ``fx -= sx``, clamped to the border (weight 0);
rows likewise; horizontal pass ``S[sx]*(1-fx) + S[sx+1]*fx`` then vertical
``H0*(1-fy) + H1*fy``, every op rounded to float32.  "parity unpinned" against cv2 itself
(its SIMD builds may fuse the vertical multiply-add; see tlod/data/blob.py).
"""
import numpy as np
import torch
from PIL import Image

PIXEL_MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])


def imread_rgb(path):
    a = np.asarray(Image.open(path).convert("RGB"))
    return a


def _coeffs(src_len, dst_len, fx):
    """resize.cpp coefficient loop for one axis: (sx, 1 - f, f) per destination index."""
    scale = 1.0 / fx
    sx = np.zeros(dst_len, np.int64)
    c0 = np.zeros(dst_len, np.float32)
    c1 = np.zeros(dst_len, np.float32)
    for d in range(dst_len):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0.0), 0
        if s >= src_len - 1:
            f, s = np.float32(0.0), src_len - 1
        sx[d], c0[d], c1[d] = s, np.float32(1.0) - f, f
    return sx, c0, c1


def cv2_resize_linear(im, fx):
    """im: H x W x C float32 -> round(H*fx) x round(W*fx) x C float32."""
    H, W, C = im.shape
    Hd, Wd = int(np.rint(H * fx)), int(np.rint(W * fx))
    sx, a0, a1 = _coeffs(W, Wd, fx)
    sy, b0, b1 = _coeffs(H, Hd, fx)
    sx1 = np.minimum(sx + 1, W - 1)
    # horizontal pass over every source row
    hrow = (im[:, sx, :] * a0[None, :, None]).astype(np.float32) + \
        (im[:, sx1, :] * a1[None, :, None]).astype(np.float32)
    hrow = hrow.astype(np.float32)
    sy1 = np.minimum(sy + 1, H - 1)
    out = (hrow[sy] * b0[:, None, None]).astype(np.float32) + \
        (hrow[sy1] * b1[:, None, None]).astype(np.float32)
    return out.astype(np.float32)


def prep_im_for_blob(im, pixel_means, target_size):
    """blob.py:35-52 (MAX_SIZE not applied, :44-46 commented out)."""
    im = im.astype(np.float32, copy=False)
    im -= pixel_means
    im_scale = float(target_size) / float(np.min(im.shape[0:2]))
    return cv2_resize_linear(im, im_scale), im_scale


def get_minibatch(entry, scales=(600,), use_all_gt=True):
    """minibatch.py:19-57 + _get_image_blob :59-82, one image; returns the blobs dict."""
    random_scale_inds = np.random.randint(0, high=len(scales), size=1)
    im = imread_rgb(entry["image"])
    im = im[:, :, ::-1]
    if entry["flipped"]:
        im = im[:, ::-1, :]
    im, im_scale = prep_im_for_blob(np.array(im), PIXEL_MEANS, scales[random_scale_inds[0]])
    blob = im[None].astype(np.float32)
    gt_inds = np.where(entry["gt_classes"] != 0)[0]
    gt_boxes = np.empty((len(gt_inds), 5), dtype=np.float32)
    gt_boxes[:, 0:4] = entry["boxes"][gt_inds, :] * im_scale
    gt_boxes[:, 4] = entry["gt_classes"][gt_inds]
    need = np.zeros((1,), np.float32) if entry["image"].find("source_") == -1 else \
        np.ones((1,), np.float32)
    return {"data": blob, "gt_boxes": gt_boxes, "need_backprop": need,
            "im_info": np.array([[blob.shape[1], blob.shape[2], im_scale]], dtype=np.float32)}


def roibatch_item(entry, ratio, training, max_num_box):
    """roibatchLoader.__getitem__ (roibatchLoader.py:58-229) for one roidb entry whose
    group target ratio is ``ratio`` (a float32 tensor element, as the reference stores
    it).  Returns (data CHW, im_info (3,), gt_boxes, num_boxes, need_backprop)."""
    blobs = get_minibatch(entry)
    data = torch.from_numpy(blobs["data"])
    im_info = torch.from_numpy(blobs["im_info"])
    data_height, data_width = data.size(1), data.size(2)
    if not training:
        data = data.permute(0, 3, 1, 2).contiguous().view(3, data_height, data_width)
        return data, im_info.view(3), torch.FloatTensor([1, 1, 1, 1, 1]), 0, 0.0
    np.random.shuffle(blobs["gt_boxes"])
    gt_boxes = torch.from_numpy(blobs["gt_boxes"])
    ratio = torch.tensor(ratio, dtype=torch.float32)
    if entry["need_crop"]:
        if ratio < 1:
            min_y = int(torch.min(gt_boxes[:, 1]))
            max_y = int(torch.max(gt_boxes[:, 3]))
            trim_size = int(np.floor(data_width / ratio))
            if trim_size > data_height:
                trim_size = data_height
            box_region = max_y - min_y + 1
            if min_y == 0:
                y_s = 0
            else:
                if (box_region - trim_size) < 0:
                    y_s_min = max(max_y - trim_size, 0)
                    y_s_max = min(min_y, data_height - trim_size)
                    y_s = y_s_min if y_s_min == y_s_max else \
                        np.random.choice(range(y_s_min, y_s_max))
                else:
                    y_s_add = int((box_region - trim_size) / 2)
                    y_s = min_y if y_s_add == 0 else np.random.choice(range(min_y, min_y + y_s_add))
            data = data[:, y_s:(y_s + trim_size), :, :]
            gt_boxes[:, 1] = gt_boxes[:, 1] - float(y_s)
            gt_boxes[:, 3] = gt_boxes[:, 3] - float(y_s)
            gt_boxes[:, 1].clamp_(0, trim_size - 1)
            gt_boxes[:, 3].clamp_(0, trim_size - 1)
        else:
            min_x = int(torch.min(gt_boxes[:, 0]))
            max_x = int(torch.max(gt_boxes[:, 2]))
            trim_size = int(np.ceil(data_height * ratio))
            if trim_size > data_width:
                trim_size = data_width
            box_region = max_x - min_x + 1
            if min_x == 0:
                x_s = 0
            else:
                if (box_region - trim_size) < 0:
                    x_s_min = max(max_x - trim_size, 0)
                    x_s_max = min(min_x, data_width - trim_size)
                    x_s = x_s_min if x_s_min == x_s_max else \
                        np.random.choice(range(x_s_min, x_s_max))
                else:
                    x_s_add = int((box_region - trim_size) / 2)
                    x_s = min_x if x_s_add == 0 else np.random.choice(range(min_x, min_x + x_s_add))
            data = data[:, :, x_s:(x_s + trim_size), :]
            gt_boxes[:, 0] = gt_boxes[:, 0] - float(x_s)
            gt_boxes[:, 2] = gt_boxes[:, 2] - float(x_s)
            gt_boxes[:, 0].clamp_(0, trim_size - 1)
            gt_boxes[:, 2].clamp_(0, trim_size - 1)
    if ratio < 1:
        padding_data = torch.zeros(int(np.ceil(data_width / ratio)), data_width, 3)
        padding_data[:data_height, :, :] = data[0]
        im_info[0, 0] = padding_data.size(0)
    elif ratio > 1:
        padding_data = torch.zeros(data_height, int(np.ceil(data_height * ratio)), 3)
        padding_data[:, :data_width, :] = data[0]
        im_info[0, 1] = padding_data.size(1)
    else:
        trim_size = min(data_height, data_width)
        padding_data = data[0][:trim_size, :trim_size, :]
        gt_boxes[:, :4].clamp_(0, trim_size)
        im_info[0, 0] = trim_size
        im_info[0, 1] = trim_size
    not_keep = (gt_boxes[:, 0] == gt_boxes[:, 2]) | (gt_boxes[:, 1] == gt_boxes[:, 3])
    keep = torch.nonzero(not_keep == 0).view(-1)
    gt_boxes_padding = torch.zeros(max_num_box, gt_boxes.size(1))
    if keep.numel() != 0:
        gt_boxes = gt_boxes[keep]
        num_boxes = min(gt_boxes.size(0), max_num_box)
        gt_boxes_padding[:num_boxes, :] = gt_boxes[:num_boxes]
    else:
        num_boxes = 0
    padding_data = padding_data.permute(2, 0, 1).contiguous()
    return padding_data, im_info.view(3), gt_boxes_padding, num_boxes, \
        float(blobs["need_backprop"][0])
