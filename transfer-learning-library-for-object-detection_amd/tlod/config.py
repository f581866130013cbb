"""Configuration mirror of ``model.utils.config.cfg`` (lib/model/utils/config.py:11-305).

Only the keys the training hot path reads are mirrored, with the reference defaults.
``cfg`` is an attribute-dict like the reference's EasyDict so reference-style code reads
``cfg.TRAIN.RPN_PRE_NMS_TOP_N``; the ops themselves take explicit values (no hidden
global reads inside kernels).  ``cfg_from_file`` uses yaml.safe_load (the reference's
bare ``yaml.load`` breaks on PyYAML >= 6, config.py:373-379).
"""
import ast
import copy

import numpy as np
import yaml


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __deepcopy__(self, memo):
        return AttrDict({k: copy.deepcopy(v, memo) for k, v in self.items()})


def _defaults():
    C = AttrDict()
    C.TRAIN = AttrDict(
        LEARNING_RATE=0.001, MOMENTUM=0.9, WEIGHT_DECAY=0.0005, GAMMA=0.1, DOUBLE_BIAS=True,
        TRUNCATED=False, BIAS_DECAY=False, SCALES=(600,), MAX_SIZE=1000, IMS_PER_BATCH=1,
        BATCH_SIZE=128, FG_FRACTION=0.25, FG_THRESH=0.5, BG_THRESH_HI=0.5, BG_THRESH_LO=0.1,
        USE_FLIPPED=True, BBOX_REG=True, BBOX_THRESH=0.5, BBOX_NORMALIZE_TARGETS=True,
        BBOX_INSIDE_WEIGHTS=(1.0, 1.0, 1.0, 1.0), BBOX_NORMALIZE_TARGETS_PRECOMPUTED=True,
        BBOX_NORMALIZE_MEANS=(0.0, 0.0, 0.0, 0.0), BBOX_NORMALIZE_STDS=(0.1, 0.1, 0.2, 0.2),
        PROPOSAL_METHOD="gt", HAS_RPN=True, RPN_POSITIVE_OVERLAP=0.7, RPN_NEGATIVE_OVERLAP=0.3,
        RPN_CLOBBER_POSITIVES=False, RPN_FG_FRACTION=0.5, RPN_BATCHSIZE=256,
        RPN_NMS_THRESH=0.7, RPN_PRE_NMS_TOP_N=12000, RPN_POST_NMS_TOP_N=2000, RPN_MIN_SIZE=8,
        RPN_BBOX_INSIDE_WEIGHTS=(1.0, 1.0, 1.0, 1.0), RPN_POSITIVE_WEIGHT=-1.0,
        USE_ALL_GT=True, BN_TRAIN=False, DISPLAY=10)
    C.TEST = AttrDict(
        SCALES=(600,), MAX_SIZE=1000, NMS=0.3, BBOX_REG=True, HAS_RPN=False,
        RPN_NMS_THRESH=0.7, RPN_PRE_NMS_TOP_N=6000, RPN_POST_NMS_TOP_N=300, RPN_MIN_SIZE=16,
        MODE="nms")
    C.RESNET = AttrDict(MAX_POOL=False, FIXED_BLOCKS=1)
    C.PIXEL_MEANS = np.array([[[102.9801, 115.9465, 122.7717]]])
    C.RNG_SEED = 3
    C.EPS = 1e-14
    C.USE_GPU_NMS = True
    C.POOLING_MODE = "crop"
    C.POOLING_SIZE = 7
    C.MAX_NUM_GT_BOXES = 20
    C.ANCHOR_SCALES = [4, 8, 16, 32]
    C.ANCHOR_RATIOS = [0.5, 1, 2]
    C.FEAT_STRIDE = [16]
    C.CUDA = False
    C.CROP_RESIZE_WITH_MAX_POOL = True
    return C


cfg = _defaults()


def reset_cfg():
    cfg.clear()
    cfg.update(_defaults())


def _merge(a, b):
    for k, v in a.items():
        if k not in b:
            raise KeyError(f"{k} is not a valid config key")
        if isinstance(v, dict):
            _merge(v, b[k])
        else:
            old = b[k]
            if isinstance(old, np.ndarray):
                v = np.array(v, dtype=old.dtype)
            elif isinstance(old, tuple) and isinstance(v, list):
                v = tuple(v)
            b[k] = v


def cfg_from_file(filename):
    """config.py:373-379 (safe YAML)."""
    with open(filename) as f:
        y = yaml.safe_load(f) or {}
    y.pop("EXP_DIR", None)
    _merge(y, cfg)


def cfg_from_list(cfg_list):
    """config.py:382-402: ['KEY.SUB', 'value', ...]."""
    assert len(cfg_list) % 2 == 0
    for k, v in zip(cfg_list[0::2], cfg_list[1::2]):
        d = cfg
        keys = k.split(".")
        for sub in keys[:-1]:
            d = d[sub]
        try:
            val = ast.literal_eval(v)
        except (ValueError, SyntaxError):
            val = v
        d[keys[-1]] = val


# cfgs/vgg16.yml and cfgs/res101.yml (the two configs the hot path trains with)
VGG16_YML = {"TRAIN": {"HAS_RPN": True, "BBOX_NORMALIZE_TARGETS_PRECOMPUTED": True,
                       "RPN_POSITIVE_OVERLAP": 0.7, "RPN_BATCHSIZE": 256, "PROPOSAL_METHOD": "gt",
                       "BG_THRESH_LO": 0.0, "BATCH_SIZE": 256, "LEARNING_RATE": 0.01},
             "TEST": {"HAS_RPN": True}, "POOLING_MODE": "align",
             "CROP_RESIZE_WITH_MAX_POOL": False}
RES101_YML = {"TRAIN": {"HAS_RPN": True, "BBOX_NORMALIZE_TARGETS_PRECOMPUTED": True,
                        "RPN_POSITIVE_OVERLAP": 0.7, "RPN_BATCHSIZE": 256, "PROPOSAL_METHOD": "gt",
                        "BG_THRESH_LO": 0.0, "DISPLAY": 20, "BATCH_SIZE": 128,
                        "WEIGHT_DECAY": 0.0001, "DOUBLE_BIAS": False, "LEARNING_RATE": 0.001},
              "TEST": {"HAS_RPN": True}, "POOLING_SIZE": 7, "POOLING_MODE": "align",
              "CROP_RESIZE_WITH_MAX_POOL": False}


# per-dataset set_cfgs of the training drivers (methods/faster_rcnn/faster_rcnn_train.py:
# 155-175, methods/DAF/DAF_train.py:168-198)
DATASET_CFGS = {
    "pascal_voc": ["ANCHOR_SCALES", "[8, 16, 32]", "ANCHOR_RATIOS", "[0.5,1,2]",
                   "MAX_NUM_GT_BOXES", "20"],
    "cityscape": ["ANCHOR_SCALES", "[4,8,16,32]", "ANCHOR_RATIOS", "[0.5,1,2]",
                  "MAX_NUM_GT_BOXES", "50"],
}


def setup_training_cfg(net="vgg16", dataset="cityscape"):
    """What the drivers do for --net vgg16|res101 --dataset cityscape|pascal_voc: cfgs/<net>.yml
    then the dataset's set_cfgs."""
    reset_cfg()
    _merge(copy.deepcopy(VGG16_YML if net == "vgg16" else RES101_YML), cfg)
    cfg_from_list(DATASET_CFGS[dataset])
    return cfg
