"""Data layer host logic on the CPU: the VOC reader (lib/datasets/pascal_voc.py), roidb
preparation (lib/roi_data_layer/roidb.py), the cv::resize INTER_LINEAR tables of the
device blob (tlod/data/blob.py) and the crop / pad / gt plan of roibatchLoader, against the
oracle restatement (oracle/blob.py) and hand-computed values."""
import os

import numpy as np
import pytest

from oracle import blob as oblob
from tlod.config import cfg, setup_training_cfg
from tlod.data import blob as tblob
from tlod.data.imdb import VOC_CLASSES, pascal_voc
from tlod.data.loader import roibatchLoader
from tlod.data.roidb import combined_roidb
from tlod.data.synthetic import write_voc

SIZES = [(120, 160), (100, 260), (90, 40), (64, 64), (150, 100)]  # incl. ratio > 2 and < 0.5


def _dataset(root):
    rng = np.random.default_rng(0)
    images = []
    for i, (H, W) in enumerate(SIZES):
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        objs = []
        for k in range(3):
            x1 = int(rng.integers(1, W // 2))
            y1 = int(rng.integers(1, H // 2))
            objs.append((VOC_CLASSES[1 + (i + k) % 20], x1, y1,
                         int(rng.integers(x1 + 4, W + 1)), int(rng.integers(y1 + 4, H + 1)), k == 2))
        images.append((("source_" if i % 2 == 0 else "target_") + f"{i:04d}", img, objs))
    write_voc(str(root), images)
    return images


def test_voc_reader_and_flip(tmp_path):
    images = _dataset(tmp_path)
    db = pascal_voc("trainval", "2007", str(tmp_path))
    assert db.num_images == len(SIZES) and db.image_index[1] == "target_0001"
    r = db.roidb[0]
    name, x1, y1, x2, y2, diff = images[0][2][0]
    assert r["boxes"].dtype == np.uint16
    assert list(r["boxes"][0]) == [x1 - 1, y1 - 1, x2 - 1, y2 - 1]   # pascal_voc.py:250-253
    assert r["gt_classes"][0] == VOC_CLASSES.index(name) and r["gt_ishard"][2] == 1
    assert r["gt_overlaps"][0, VOC_CLASSES.index(name)] == 1.0
    assert r["seg_areas"][0] == (x2 - x1 + 1) * (y2 - y1 + 1)
    db.append_flipped_images()
    W = SIZES[0][1]
    f = db.roidb[len(SIZES)]
    assert f["flipped"] and db.num_images == 2 * len(SIZES)
    assert list(f["boxes"][0]) == [W - (x2 - 1) - 1, y1 - 1, W - (x1 - 1) - 1, y2 - 1]


def test_combined_roidb_ratio_ranking(tmp_path):
    _dataset(tmp_path)
    setup_training_cfg("vgg16", "pascal_voc")
    cfg.TRAIN.USE_FLIPPED = True
    _, roidb, ratio_list, ratio_index = combined_roidb("voc_2007_trainval", str(tmp_path))
    assert len(roidb) == 2 * len(SIZES)
    ratios = [min(max(W / H, 0.5), 2.0) for H, W in SIZES] * 2
    np.testing.assert_array_equal(ratio_list, np.sort(ratios))
    np.testing.assert_array_equal(ratio_index, np.argsort(ratios))
    crop = [r["need_crop"] for r in roidb]
    assert crop == [int(W / H > 2 or W / H < 0.5) for H, W in SIZES] * 2
    assert all(os.path.exists(r["image"]) for r in roidb)


@pytest.mark.parametrize("src,fx", [(37, 600 / 37), (1024, 600 / 1024), (500, 1.2), (600, 1.0),
                                    (1200, 0.5), (333, 600 / 333)])
def test_linear_taps_match_oracle_coefficients(src, fx):
    dst = tblob.resized_size(src, fx)
    assert dst == int(np.rint(src * fx))
    t = tblob.linear_taps(src, dst, fx)
    sx, c0, c1 = oblob._coeffs(src, dst, fx)
    np.testing.assert_array_equal(t["i0"], sx)
    np.testing.assert_array_equal(t["i1"], np.minimum(sx + 1, src - 1))
    np.testing.assert_array_equal(t["w0"], c0)
    np.testing.assert_array_equal(t["w1"], c1)
    tf = tblob.linear_taps(src, dst, fx, flip=True)
    np.testing.assert_array_equal(tf["i0"], src - 1 - t["i0"])


def _kernel_emulation(img_rgb, fx, flip):
    """The device kernel's arithmetic (csrc/blob.hip) in numpy float32."""
    H, W, _ = img_rgb.shape
    lut = tblob.pixel_lut(cfg.PIXEL_MEANS)
    Hr, Wr = tblob.resized_size(H, fx), tblob.resized_size(W, fx)
    xt, yt = tblob.linear_taps(W, Wr, fx, flip), tblob.linear_taps(H, Hr, fx)
    out = np.zeros((3, Hr, Wr), np.float32)
    for c in range(3):
        S = lut[c][img_rgb[:, :, 2 - c]]
        h = S[:, xt["i0"]] * xt["w0"] + S[:, xt["i1"]] * xt["w1"]
        out[c] = h[yt["i0"]] * yt["w0"][:, None] + h[yt["i1"]] * yt["w1"][:, None]
    return out


@pytest.mark.parametrize("fx,flip", [(1.25, False), (0.7, True), (1.0, False), (600 / 37, True)])
def test_blob_arithmetic_matches_oracle(fx, flip):
    """pixel LUT (numpy's float32 -= float64) + taps reproduce the oracle's prep_im_for_blob
    bit for bit."""
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    got = _kernel_emulation(img, fx, flip)
    im = img[:, :, ::-1]
    if flip:
        im = im[:, ::-1, :]
    im = np.array(im).astype(np.float32)
    im -= oblob.PIXEL_MEANS  # blob.py:38-39: in place, float32 result
    ref = oblob.cv2_resize_linear(im, fx)
    np.testing.assert_array_equal(got, ref.astype(np.float32).transpose(2, 0, 1))


def test_loader_plan_matches_oracle(tmp_path):
    """roibatchLoader's host plan (RNG draws, crop / pad geometry, gt bookkeeping,
    im_info, need_backprop) equals the oracle's literal restatement, item by item."""
    _dataset(tmp_path)
    setup_training_cfg("vgg16", "pascal_voc")
    cfg.TRAIN.USE_FLIPPED = True
    imdb, roidb, ratio_list, ratio_index = combined_roidb("voc_2007_trainval", str(tmp_path))
    for training in (True, False):
        ld = roibatchLoader(roidb, ratio_list, ratio_index, 1, imdb.num_classes,
                            training=training, with_need_backprop=True)
        for idx in range(len(roidb)):
            np.random.seed(100 + idx)
            p = ld.plan(idx)
            entry = roidb[int(ratio_index[idx]) if training else idx]
            np.random.seed(100 + idx)
            data, im_info, gt, num, need = oblob.roibatch_item(
                entry, ld.ratio_list_batch[idx], training, cfg.MAX_NUM_GT_BOXES)
            assert tuple(data.shape[1:]) == p["out"], (idx, data.shape, p)
            np.testing.assert_array_equal(p["im_info"], im_info.numpy())
            np.testing.assert_array_equal(p["gt_boxes"], gt.numpy())
            assert p["num_boxes"] == num and p["need_backprop"] == need
            # the oracle's blob where the plan keeps data, zeros elsewhere
            y0, x0 = p["crop"]
            Hd, Wd = p["keep"]
            d = data.numpy()
            assert not d[:, Hd:, :].any() and not d[:, :, Wd:].any()
            ref = _kernel_emulation(p["img"], p["im_scale"], p["flip"])
            np.testing.assert_array_equal(d[:, :Hd, :Wd], ref[:, y0:y0 + Hd, x0:x0 + Wd])
