"""Training roidb preparation (lib/roi_data_layer/roidb.py, same in lib/DAF/roidb.py)."""
import numpy as np
from PIL import Image

from ..config import cfg
from .imdb import get_imdb


def prepare_roidb(imdb):
    """roidb.py:14-48: image path / id / size and the max-overlap class of each box."""
    roidb = imdb.roidb
    sizes = [Image.open(imdb.image_path_at(i)).size for i in range(imdb.num_images)]
    for i in range(len(imdb.image_index)):
        r = roidb[i]
        r["img_id"] = imdb.image_id_at(i)
        r["image"] = imdb.image_path_at(i)
        r["width"], r["height"] = sizes[i]
        gt = np.asarray(r["gt_overlaps"])
        r["max_classes"] = gt.argmax(axis=1)
        r["max_overlaps"] = gt.max(axis=1)
        assert all(r["max_classes"][r["max_overlaps"] == 0] == 0)
        assert all(r["max_classes"][r["max_overlaps"] > 0] != 0)


def rank_roidb_ratio(roidb):
    """roidb.py:51-74: width / height clamped to [0.5, 2] (need_crop when clamped);
    returns the sorted ratios and the sorting permutation."""
    ratio_large, ratio_small = 2, 0.5
    ratio_list = []
    for r in roidb:
        ratio = r["width"] / float(r["height"])
        if ratio > ratio_large:
            r["need_crop"], ratio = 1, ratio_large
        elif ratio < ratio_small:
            r["need_crop"], ratio = 1, ratio_small
        else:
            r["need_crop"] = 0
        ratio_list.append(ratio)
    ratio_list = np.array(ratio_list)
    ratio_index = np.argsort(ratio_list)
    return ratio_list[ratio_index], ratio_index


def filter_roidb(roidb):
    """roidb.py:76-87: drop images without boxes."""
    return [r for r in roidb if len(r["boxes"]) != 0]


def combined_roidb(imdb_names, devkit_path, training=True, classes=None):
    """roidb.py:89-130 -> (imdb, roidb, ratio_list, ratio_index).  Flipped copies are
    appended when cfg.TRAIN.USE_FLIPPED (the training drivers set it True)."""
    def get_roidb(name):
        imdb = get_imdb(name, devkit_path, classes)
        if cfg.TRAIN.USE_FLIPPED:
            imdb.append_flipped_images()
        prepare_roidb(imdb)
        return imdb, imdb.roidb

    pairs = [get_roidb(s) for s in imdb_names.split("+")]
    imdb, roidb = pairs[0][0], list(pairs[0][1])
    for _, r in pairs[1:]:
        roidb.extend(r)
    if training:
        roidb = filter_roidb(roidb)
    ratio_list, ratio_index = rank_roidb_ratio(roidb)
    return imdb, roidb, ratio_list, ratio_index
