"""BASELINE config 1 — methods/faster_rcnn source-only VGG16, bs=1, one synthetic
600x1000 VOC-format image — through the device data layer and the source-only detector,
against the CPU oracle (oracle/blob.py, oracle/frcnn_step.py).

  * the data layer (VOC XML + ImageSets reader, roidb with flips and aspect ranking,
    roibatchLoader crop / pad / gt padding, the device image blob) equals the oracle's
    literal restatement bit for bit, item by item;
  * one training step from that VOC directory: every loss within 1e-4 of the oracle, the
    sampled RoIs identical (replayed numpy draws), every gradient within 2x the error of the
    reference's own fp32 arithmetic (tests/helpers.pattern_grad_bar);
  * eval mode returns the TEST proposals and per-class outputs (faster_rcnn.py:62-115).
"""
import numpy as np
import pytest
import torch

from helpers import arm_device_taps, pattern_grad_bar, record_pattern

pytestmark = pytest.mark.gpu
dev = "cuda"


def _setup(root, sizes, seed, training=True):
    from tlod.config import cfg, setup_training_cfg
    from tlod.data.imdb import VOC_CLASSES
    from tlod.data.loader import roibatchLoader
    from tlod.data.roidb import combined_roidb
    from tlod.data.synthetic import synthetic_voc
    synthetic_voc(str(root), sizes, VOC_CLASSES, seed=seed, n_objects=6)
    setup_training_cfg("vgg16", "pascal_voc")
    cfg.TRAIN.USE_FLIPPED = True
    imdb, roidb, ratio_list, ratio_index = combined_roidb("voc_2007_trainval", str(root))
    return imdb, roidb, ratio_index, roibatchLoader(roidb, ratio_list, ratio_index, 1,
                                                    imdb.num_classes, training=training,
                                                    with_need_backprop=True)


@pytest.mark.parametrize("training", [True, False])
def test_loader_items_match_oracle(tmp_path, training):
    from oracle import blob as oblob
    from tlod.config import cfg
    sizes = [(375, 500), (333, 900), (480, 200), (256, 256)]
    _, roidb, ratio_index, ld = _setup(tmp_path, sizes, seed=5, training=training)
    for idx in range(len(roidb)):
        np.random.seed(7 + idx)
        data, im_info, gt, num, need = ld[idx]
        torch.cuda.synchronize()
        entry = roidb[int(ratio_index[idx]) if training else idx]
        np.random.seed(7 + idx)
        rd, ri, rg, rn, rneed = oblob.roibatch_item(entry, ld.ratio_list_batch[idx], training,
                                                    cfg.MAX_NUM_GT_BOXES)
        assert data.shape == rd.shape, (idx, data.shape, rd.shape)
        np.testing.assert_array_equal(data.cpu().numpy(), rd.numpy())
        np.testing.assert_array_equal(im_info.cpu().numpy(), ri.numpy())
        np.testing.assert_array_equal(gt.cpu().numpy(), rg.numpy())
        assert int(num) == rn and float(need[0]) == rneed


def test_source_only_vgg16_step_config1(tmp_path):
    """BASELINE.json configs[0]: one source-only step on one 600x1000 VOC-format image."""
    from oracle.frcnn_step import OracleFRCNN
    from oracle.frcnn_step import total_loss as o_total
    from tlod.data.imdb import VOC_CLASSES
    from tlod.data.loader import collate
    from tlod.detector.train import build_model, make_optimizer, train_step
    imdb, roidb, ratio_index, ld = _setup(tmp_path, [(600, 1000)], seed=3)
    m = build_model("faster_rcnn", dev, "vgg16", classes=VOC_CLASSES, dataset="pascal_voc")
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    np.random.seed(3)  # cfg.RNG_SEED (faster_rcnn_train.py:187)
    data, im_info, gt, num, _ = collate([ld[0]])
    assert tuple(data.shape) == (1, 3, 600, 1000)
    m.replay_rng = np.random.RandomState(3)
    m.capture = {}
    taps = arm_device_taps(m)
    out = m(data, im_info, gt, num)
    loss = m.total_loss(out)
    loss.backward()
    torch.cuda.synchronize()

    o = OracleFRCNN(len(VOC_CLASSES), scales=(8, 16, 32), dropout=0.0).train()
    o.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=True)
    cpu = (data.cpu(), im_info.cpu(), gt.cpu())
    s_rois = m.capture["s_rois"].cpu().numpy()
    box = {}

    def run32():
        box["ref"] = o(*cpu, np.random.RandomState(3), rois_override=s_rois)
        o_total(box["ref"]).backward()
    own = record_pattern(o, run32)
    ref = box["ref"]
    names = ["rpn_loss_cls", "rpn_loss_box", "RCNN_loss_cls", "RCNN_loss_bbox"]
    for name, i in zip(names, [3, 4, 5, 6]):
        g, r = float(out[i].detach()), float(ref[name].detach())
        assert abs(g - r) <= 1e-4 * max(abs(r), 1e-3), (name, g, r)
    np.testing.assert_array_equal(out[0].cpu().numpy().reshape(-1, 5), ref["rois"].reshape(-1, 5))
    np.testing.assert_array_equal(out[7].cpu().numpy(), ref["labels"].numpy())

    pattern_grad_bar(m, o, lambda mod, b: o_total(mod(*b, np.random.RandomState(3),
                                                      rois_override=s_rois)),
                     cpu, taps, None, own)

    # and a full step (clip_gradient(10) + SGD) trains
    opt = make_optimizer(m, 1e-3)
    for _ in range(2):
        v = float(train_step(m, opt, (data, im_info, gt, num)))
        assert np.isfinite(v)


def test_source_only_eval_outputs(tmp_path):
    from tlod.data.imdb import VOC_CLASSES
    from tlod.data.loader import collate
    from tlod.detector.train import build_model
    _, _, _, ld = _setup(tmp_path, [(600, 1000)], seed=4, training=False)
    m = build_model("faster_rcnn", dev, "vgg16", classes=VOC_CLASSES, dataset="pascal_voc").eval()
    data, im_info, gt, num, _ = collate([ld[0]])
    with torch.no_grad():
        rois, cls_prob, bbox_pred, l1, l2, l3, l4, lab = m(data, im_info, gt, num)
    assert rois.shape == (1, 300, 5) and cls_prob.shape == (1, 300, 21)
    assert bbox_pred.shape == (1, 300, 84) and lab is None
    assert (l1, l2, l3, l4) == (0, 0, 0, 0)
    torch.testing.assert_close(cls_prob.sum(-1), torch.ones(1, 300, device=dev))
