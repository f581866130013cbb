"""Test-time detections (tlod_detect_f32: de-normalise, decode, clip, rescale, per-class
sort + NMS in one launch) against the oracle restatement of methods/DAF/DAF_test.py:279-333,
and the whole test loop on a synthetic VOC set down to VOC AP."""
import numpy as np
import pytest
import torch

from helpers import clustered_boxes

pytestmark = pytest.mark.gpu
dev = "cuda"


def _inputs(rng, R, C, agnostic):
    b = clustered_boxes(rng, R, W=1000, H=600, clusters=25)
    rois = np.concatenate([np.zeros((R, 1), np.float32), b], 1)
    logits = rng.normal(0, 2, (R, C)).astype(np.float32)
    e = np.exp(logits - logits.max(1, keepdims=True))
    prob = (e / e.sum(1, keepdims=True)).astype(np.float32)
    bp = rng.normal(0, 0.5, (R, 4 if agnostic else 4 * C)).astype(np.float32)
    return rois, prob, bp


@pytest.mark.parametrize("R,C,agnostic,thresh", [(300, 21, False, 0.0), (300, 9, False, 0.05),
                                                 (2000, 9, False, 0.0), (300, 21, True, 0.0),
                                                 (17, 3, False, 0.5)])
def test_detect_matches_oracle(R, C, agnostic, thresh):
    from oracle import detect as odet
    from tlod.config import setup_training_cfg
    from tlod.eval.detect import detect
    setup_training_cfg("vgg16", "pascal_voc")
    rng = np.random.default_rng(R + C)
    rois, prob, bp = _inputs(rng, R, C, agnostic)
    info = np.array([600, 1000, 1.6], np.float32)
    dets, counts, boxes = detect(torch.from_numpy(rois).to(dev), torch.from_numpy(prob).to(dev),
                                 torch.from_numpy(bp).to(dev), torch.from_numpy(info).to(dev),
                                 agnostic, thresh, 0.3, return_boxes=True)
    boxes = boxes.cpu().numpy()
    ref_boxes = odet.decode(rois, bp, info, C, agnostic)
    np.testing.assert_allclose(boxes[:, 1:], ref_boxes[:, 1:], rtol=2e-6, atol=1e-4)
    # per-class threshold / sort / NMS bit-exact given the device-decoded boxes
    ref = odet.postprocess(boxes, prob, thresh, 0.3, max_per_image=0)
    d, n = dets.cpu().numpy(), counts.cpu().numpy()
    assert n[0] == 0
    for j in range(1, C):
        np.testing.assert_array_equal(d[j, :n[j]], ref[j], err_msg=f"class {j}")
    assert sum(int(x) for x in n[1:]) > 0


def test_eval_loop_on_synthetic_voc(tmp_path):
    """The eval driver end to end: test roibatchLoader -> eval-mode source-only VGG16 ->
    tlod_detect_f32 -> max_per_image -> comp4 files -> VOC AP; the same all_boxes as the
    oracle post-processing of the same model outputs."""
    from oracle import detect as odet
    from tlod.config import cfg
    from tlod.data.imdb import VOC_CLASSES, pascal_voc
    from tlod.data.loader import roibatchLoader
    from tlod.data.roidb import prepare_roidb, rank_roidb_ratio
    from tlod.data.synthetic import synthetic_voc
    from tlod.detector.train import build_model
    from tlod.eval.detect import detect, eval_net, limit_per_image
    synthetic_voc(str(tmp_path), [(375, 500), (500, 333), (600, 800)], VOC_CLASSES, seed=9,
                  n_objects=4, prefix="target_", image_set="test")
    m = build_model("faster_rcnn", dev, "vgg16", classes=VOC_CLASSES, dataset="pascal_voc").eval()
    imdb = pascal_voc("test", "2007", str(tmp_path))
    prepare_roidb(imdb)
    ratio_list, ratio_index = rank_roidb_ratio(imdb.roidb)
    ld = roibatchLoader(imdb.roidb, ratio_list, ratio_index, 1, imdb.num_classes, training=False)
    aps, all_boxes = eval_net(m, imdb, ld, str(tmp_path / "out"))
    assert set(aps) == set(VOC_CLASSES[1:]) | {"mAP"}
    assert all(0.0 <= v <= 1.0 or np.isnan(v) for v in aps.values())
    for i in range(imdb.num_images):
        data, im_info, gt, num = (t.unsqueeze(0) for t in ld[i])
        with torch.no_grad():
            rois, prob, bp = m(data, im_info, gt, num)[:3]
        _, _, boxes = detect(rois[0], prob[0], bp[0], im_info[0], return_boxes=True)
        ref = odet.postprocess(boxes.cpu().numpy(), prob[0].cpu().numpy(), 0.0,
                               cfg.TEST.NMS, max_per_image=100)
        for j in range(1, imdb.num_classes):
            np.testing.assert_array_equal(all_boxes[j][i], ref[j])
        assert sum(len(all_boxes[j][i]) for j in range(1, imdb.num_classes)) <= 100 + 20
    _ = limit_per_image
