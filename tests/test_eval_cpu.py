"""VOC evaluation (lib/datasets/voc_eval.py, pascal_voc.py:276-356) pinned by a
hand-computed fixture, and the max_per_image cut (methods/DAF/DAF_test.py:323-333)."""
import numpy as np
import pytest

from tlod.data.imdb import pascal_voc
from tlod.data.synthetic import write_voc
from tlod.eval.detect import limit_per_image
from tlod.eval.voc import voc_ap

CLASSES = ("__background__", "car", "bus")


def _fixture(root):
    """image a: cars G1 = [1,1,10,10], G2 = [21,21,30,30]; image b: a difficult car G3 =
    [1,1,10,10] and a bus [5,5,40,40] (1-based VOC coordinates)."""
    z = np.zeros((48, 48, 3), np.uint8)
    write_voc(str(root), [("a", z, [("car", 1, 1, 10, 10, 0), ("car", 21, 21, 30, 30, 0)]),
                          ("b", z, [("car", 1, 1, 10, 10, 1), ("bus", 5, 5, 40, 40, 0)])],
              image_set="test")
    return pascal_voc("test", "2007", str(root), CLASSES)


def _dets():
    """0-based detections (the results writer adds 1).  By confidence, car: d1 a .9 = G1
    (TP), d2 b .8 = G3 (difficult: ignored), d3 a .7 = G1 again (FP, already detected),
    d4 a .6 = G2 (TP), d5 a .5 far away (FP).  npos = 2 ->
        tp = [1,1,1,2,2], fp = [0,0,1,1,2], rec = [.5,.5,.5,1,1], prec = [1,1,.5,2/3,.5]
        area AP = .5 * 1 + .5 * 2/3 = 5/6;  VOC07 11-point = (6 * 1 + 5 * 2/3) / 11 = 28/33.
    bus: one TP at .4 (IoU 1) -> AP 1."""
    g = lambda b, s: [b[0] - 1, b[1] - 1, b[2] - 1, b[3] - 1, s]  # noqa: E731
    car_a = np.array([g((1, 1, 10, 10), .9), g((1, 1, 10, 10), .7), g((21, 21, 30, 30), .6),
                      g((50, 50, 60, 60), .5)], np.float32)
    car_b = np.array([g((1, 1, 10, 10), .8)], np.float32)
    bus_b = np.array([g((5, 5, 40, 40), .4)], np.float32)
    empty = np.zeros((0, 5), np.float32)
    return [[[], []], [car_a, car_b], [empty, bus_b]]


@pytest.mark.parametrize("year,car_ap", [("2007", 28.0 / 33.0), ("2012", 5.0 / 6.0)])
def test_voc_eval_hand_computed(tmp_path, year, car_ap):
    imdb = _fixture(tmp_path)
    imdb._year = year  # VOC07 11-point metric for year < 2010 (pascal_voc.py:317-318)
    if year != "2007":
        import os
        os.rename(os.path.join(str(tmp_path), "VOC2007"), os.path.join(str(tmp_path), "VOC" + year))
        imdb._data_path = os.path.join(str(tmp_path), "VOC" + year)
    aps = imdb.evaluate_detections(_dets(), str(tmp_path / "out"))
    assert aps["car"] == pytest.approx(car_ap, abs=1e-12)
    assert aps["bus"] == pytest.approx(1.0, abs=1e-12)
    assert aps["mAP"] == pytest.approx((car_ap + 1.0) / 2, abs=1e-12)


def test_voc_ap_envelope():
    rec = np.array([.5, .5, .5, 1, 1])
    prec = np.array([1, 1, .5, 2 / 3, .5])
    assert voc_ap(rec, prec) == pytest.approx(5 / 6)
    assert voc_ap(rec, prec, True) == pytest.approx(28 / 33)


def test_limit_per_image():
    rng = np.random.default_rng(0)
    per = [np.zeros((0, 5), np.float32)] + [
        np.concatenate([rng.uniform(0, 100, (n, 4)), rng.uniform(0, 1, (n, 1))], 1).astype(np.float32)
        for n in (40, 50, 30)]
    out = limit_per_image(per, 100)
    allsc = np.sort(np.hstack([d[:, 4] for d in per[1:]]))
    th = allsc[-100]
    assert sum(len(d) for d in out[1:]) == int((allsc >= th).sum()) == 100
    assert all((d[:, 4] >= th).all() for d in out[1:])
    assert limit_per_image(per, 200) is per
