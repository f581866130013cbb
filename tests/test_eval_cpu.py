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


def _ap_by_detection_loop(dets, gts, ovthresh, use_07):
    """Independent statement of the VOC metric (voc_eval.py:70-211): walk the detections in
    descending confidence (np.argsort(-score), as the reference), one at a time."""
    order = np.argsort(-np.array([d[1] for d in dets]))
    used = {k: [False] * len(v) for k, v in gts.items()}
    npos = sum(1 for v in gts.values() for g in v if not g[4])
    tp, fp = [], []
    for k in order:
        img, _, box = dets[k]
        best, arg = -np.inf, -1
        for j, g in enumerate(gts[img]):
            iw = max(min(g[2], box[2]) - max(g[0], box[0]) + 1.0, 0.0)
            ih = max(min(g[3], box[3]) - max(g[1], box[1]) + 1.0, 0.0)
            inter = iw * ih
            ov = inter / ((box[2] - box[0] + 1.0) * (box[3] - box[1] + 1.0) +
                          (g[2] - g[0] + 1.0) * (g[3] - g[1] + 1.0) - inter)
            if ov > best:
                best, arg = ov, j
        t = f = 0.0
        if best > ovthresh:
            if not gts[img][arg][4]:
                if used[img][arg]:
                    f = 1.0
                else:
                    t, used[img][arg] = 1.0, True
        else:
            f = 1.0
        tp.append(t)
        fp.append(f)
    tp, fp = np.cumsum(tp), np.cumsum(fp)
    rec = tp / float(npos)
    prec = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
    return rec, prec, voc_ap(rec, prec, use_07)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_voc_eval_matches_detection_loop(tmp_path, seed):
    """tlod.eval.voc.voc_eval (per-image IoU matrices) against the per-detection loop on
    random scenes: overlapping boxes, tied scores, difficult objects, images without the
    class, detections in images without ground truth."""
    from tlod.eval.voc import voc_eval
    rng = np.random.default_rng(seed)
    z = np.zeros((8, 8, 3), np.uint8)
    images, gts, dets = [], {}, []
    for i in range(12):
        name = f"im{i:03d}"
        objs = []
        for _ in range(int(rng.integers(0, 5))):
            x1, y1 = rng.integers(1, 150, 2)
            w, h = rng.integers(5, 60, 2)
            objs.append(("car" if rng.random() < .8 else "bus", int(x1), int(y1), int(x1 + w),
                         int(y1 + h), int(rng.random() < .2)))
        images.append((name, z, objs))
        gts[name] = [o[1:] for o in objs if o[0] == "car"]
        for o in objs:  # jittered hits and duplicates, scores on a coarse grid (ties)
            for _ in range(int(rng.integers(0, 3))):
                box = np.array(o[1:5], float) + rng.normal(0, 4, 4)
                dets.append((name, float(rng.integers(0, 20)) / 20, box))
        for _ in range(int(rng.integers(0, 3))):  # false alarms
            x1, y1 = rng.uniform(1, 150, 2)
            dets.append((name, float(rng.integers(0, 20)) / 20, np.array([x1, y1, x1 + 20, y1 + 20])))
    write_voc(str(tmp_path), images, image_set="test")
    base = tmp_path / "VOC2007"
    detfile = tmp_path / "car.txt"
    with open(detfile, "w") as f:
        for name, s, b in dets:
            f.write(f"{name} {s:.3f} {b[0]:.1f} {b[1]:.1f} {b[2]:.1f} {b[3]:.1f}\n")
    dets = [(n, float(f"{s:.3f}"), np.array([float(f"{v:.1f}") for v in b])) for n, s, b in dets]
    for use_07 in (True, False):
        rec, prec, ap = voc_eval(str(detfile), str(base / "Annotations" / "{}.xml"),
                                 str(base / "ImageSets" / "Main" / "test.txt"), "car", 0.5, use_07)
        rec2, prec2, ap2 = _ap_by_detection_loop(dets, gts, 0.5, use_07)
        np.testing.assert_array_equal(rec, rec2)
        np.testing.assert_array_equal(prec, prec2)
        assert ap == ap2
    open(tmp_path / "none.txt", "w").close()  # a class without detections
    rec, prec, ap = voc_eval(str(tmp_path / "none.txt"), str(base / "Annotations" / "{}.xml"),
                             str(base / "ImageSets" / "Main" / "test.txt"), "car", 0.5, False)
    assert rec.size == 0 and prec.size == 0 and ap == 0.0
