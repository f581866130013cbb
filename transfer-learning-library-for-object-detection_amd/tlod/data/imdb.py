"""VOC-format image databases (lib/datasets/{imdb,pascal_voc,cityscape}.py).

Layout read (pascal_voc.py:91-131, cityscape.py:87-123):
    <devkit>/VOC<year>/ImageSets/Main/<image_set>.txt   one image index per line
    <devkit>/VOC<year>/Annotations/<index>.xml          PASCAL VOC objects
    <devkit>/VOC<year>/JPEGImages/<index>.jpg
``gt_roidb`` entries follow ``_load_pascal_annotation`` (pascal_voc.py:218-271): boxes are
uint16 pixel indexes made 0-based (``xmin - 1``), ``gt_overlaps`` a one-hot class matrix,
difficult objects kept (``use_diff`` handling is commented out in the reference).
``evaluate_detections`` writes the comp4 per-class results files and runs the Python VOC
AP (pascal_voc.py:276-356, tlod.eval.voc).  No pickle caches are read or written.
"""
import os
import xml.etree.ElementTree as ET

import numpy as np
from PIL import Image

VOC_CLASSES = ("__background__", "aeroplane", "bicycle", "bird", "boat", "bottle", "bus",
               "car", "cat", "chair", "cow", "diningtable", "dog", "horse", "motorbike",
               "person", "pottedplant", "sheep", "sofa", "train", "tvmonitor")
# lib/datasets/cityscape.py:51-54
CITYSCAPE_CLASSES = ("__background__", "person", "rider", "car", "truck", "bus", "train",
                     "motorcycle", "bicycle")


class imdb:
    """lib/datasets/imdb.py:22-277 (the parts the training / test drivers use)."""

    def __init__(self, name, classes=()):
        self._name = name
        self._classes = tuple(classes)
        self._image_index = []
        self._roidb = None
        self.config = {}

    @property
    def name(self):
        return self._name

    @property
    def classes(self):
        return self._classes

    @property
    def num_classes(self):
        return len(self._classes)

    @property
    def image_index(self):
        return self._image_index

    @property
    def num_images(self):
        return len(self._image_index)

    @property
    def roidb(self):
        if self._roidb is None:
            self._roidb = self.gt_roidb()
        return self._roidb

    def _get_widths(self):
        return [Image.open(self.image_path_at(i)).size[0] for i in range(self.num_images)]

    def append_flipped_images(self):
        """imdb.py:115-140: mirrored copies; x1' = w - x2 - 1 (0 when x2 >= w)."""
        widths = self._get_widths()
        for i in range(self.num_images):
            boxes = self.roidb[i]["boxes"].copy()
            oldx1, oldx2 = boxes[:, 0].copy(), boxes[:, 2].copy()
            for k in range(boxes.shape[0]):
                boxes[k, 0] = widths[i] - int(oldx2[k]) - 1 if widths[i] > oldx2[k] else 0
                boxes[k, 2] = widths[i] - int(oldx1[k]) - 1 if widths[i] > oldx1[k] else 0
            assert (boxes[:, 2] >= boxes[:, 0]).all()
            self.roidb.append({"boxes": boxes, "gt_overlaps": self.roidb[i]["gt_overlaps"],
                               "gt_classes": self.roidb[i]["gt_classes"], "flipped": True})
        self._image_index = self._image_index * 2


class pascal_voc(imdb):
    """lib/datasets/pascal_voc.py:40-393 (classes overridable for VOC-format datasets such
    as the synthetic ones of tlod.data.synthetic)."""

    def __init__(self, image_set, year, devkit_path, classes=VOC_CLASSES, prefix="voc"):
        imdb.__init__(self, f"{prefix}_{year}_{image_set}", classes)
        self._year = year
        self._image_set = image_set
        self._devkit_path = devkit_path
        self._data_path = os.path.join(devkit_path, "VOC" + year)
        self._class_to_ind = dict(zip(self.classes, range(self.num_classes)))
        self._image_ext = ".jpg"
        if not os.path.exists(self._data_path):
            raise FileNotFoundError(f"Path does not exist: {self._data_path}")
        self._image_index = self._load_image_set_index()
        self._comp_id = "comp4"
        self.config = {"cleanup": True, "use_salt": False, "use_diff": False,
                       "matlab_eval": False, "rpn_file": None, "min_size": 2}

    def image_path_at(self, i):
        return self.image_path_from_index(self._image_index[i])

    def image_id_at(self, i):
        return i

    def image_path_from_index(self, index):
        p = os.path.join(self._data_path, "JPEGImages", index + self._image_ext)
        if not os.path.exists(p):
            raise FileNotFoundError(f"Path does not exist: {p}")
        return p

    def _load_image_set_index(self):
        """pascal_voc.py:106-124: one index per line, lines of length <= 1 skipped."""
        f = os.path.join(self._data_path, "ImageSets", "Main", self._image_set + ".txt")
        if not os.path.exists(f):
            raise FileNotFoundError(f"Path does not exist: {f}")
        with open(f) as fh:
            return [x.strip() for x in fh.readlines() if len(x) > 1]

    def gt_roidb(self):
        return [self._load_pascal_annotation(i) for i in self.image_index]

    def _load_pascal_annotation(self, index):
        tree = ET.parse(os.path.join(self._data_path, "Annotations", index + ".xml"))
        objs = tree.findall("object")
        n = len(objs)
        boxes = np.zeros((n, 4), dtype=np.uint16)
        gt_classes = np.zeros((n,), dtype=np.int32)
        overlaps = np.zeros((n, self.num_classes), dtype=np.float32)
        seg_areas = np.zeros((n,), dtype=np.float32)
        ishards = np.zeros((n,), dtype=np.int32)
        for ix, obj in enumerate(objs):
            bbox = obj.find("bndbox")
            x1 = float(bbox.find("xmin").text) - 1
            y1 = float(bbox.find("ymin").text) - 1
            x2 = float(bbox.find("xmax").text) - 1
            y2 = float(bbox.find("ymax").text) - 1
            diffc = obj.find("difficult")
            ishards[ix] = 0 if diffc is None else int(diffc.text)
            cls = self._class_to_ind[obj.find("name").text.lower().strip()]
            boxes[ix, :] = [x1, y1, x2, y2]
            gt_classes[ix] = cls
            overlaps[ix, cls] = 1.0
            seg_areas[ix] = (x2 - x1 + 1) * (y2 - y1 + 1)
        return {"boxes": boxes, "gt_classes": gt_classes, "gt_ishard": ishards,
                "gt_overlaps": overlaps, "flipped": False, "seg_areas": seg_areas}

    # ------------------------------------------------------------------ evaluation
    def _results_template(self, output_dir):
        d = os.path.join(output_dir, "results", "VOC" + self._year, "Main")
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, self._comp_id + "_det_" + self._image_set + "_{:s}.txt")

    def _write_voc_results_file(self, all_boxes, output_dir):
        """pascal_voc.py:284-298: one line per detection, 1-based coordinates."""
        tmpl = self._results_template(output_dir)
        for cls_ind, cls in enumerate(self.classes):
            if cls == "__background__":
                continue
            with open(tmpl.format(cls), "wt") as f:
                for im_ind, index in enumerate(self.image_index):
                    dets = all_boxes[cls_ind][im_ind]
                    if len(dets) == 0:
                        continue
                    for k in range(dets.shape[0]):
                        f.write("{:s} {:.3f} {:.1f} {:.1f} {:.1f} {:.1f}\n".format(
                            index, dets[k, -1], dets[k, 0] + 1, dets[k, 1] + 1,
                            dets[k, 2] + 1, dets[k, 3] + 1))
        return tmpl

    def evaluate_detections(self, all_boxes, output_dir):
        """pascal_voc.py:300-356 (Python eval; VOC07 11-point metric for year < 2010).
        Returns {class: ap} plus "mAP"."""
        from ..eval.voc import voc_eval
        tmpl = self._write_voc_results_file(all_boxes, output_dir)
        annopath = os.path.join(self._data_path, "Annotations", "{:s}.xml")
        imagesetfile = os.path.join(self._data_path, "ImageSets", "Main",
                                    self._image_set + ".txt")
        use_07 = int(self._year) < 2010
        aps = {}
        for cls in self.classes:
            if cls == "__background__":
                continue
            _, _, ap = voc_eval(tmpl.format(cls), annopath, imagesetfile, cls, ovthresh=0.5,
                                use_07_metric=use_07)
            aps[cls] = float(ap)
        aps["mAP"] = float(np.mean([v for k, v in aps.items()]))
        return aps


def cityscape(image_set, year, devkit_path):
    """lib/datasets/cityscape.py:39-389: the VOC layout with the 8 Cityscapes classes."""
    return pascal_voc(image_set, year, devkit_path, CITYSCAPE_CLASSES, prefix="cityscape")


def get_imdb(name, devkit_path, classes=None):
    """lib/datasets/factory.py:24-73 for the VOC-layout names: voc_<year>_<set>,
    cityscape_<year>_<set>; a '+' joins several (combined_roidb)."""
    parts = name.split("_")
    if name.startswith("voc_") and len(parts) >= 3:
        return pascal_voc("_".join(parts[2:]), parts[1], devkit_path,
                          VOC_CLASSES if classes is None else classes)
    if name.startswith("cityscape_") and len(parts) >= 3:
        return pascal_voc("_".join(parts[2:]), parts[1], devkit_path,
                          CITYSCAPE_CLASSES if classes is None else classes, prefix="cityscape")
    raise KeyError(f"Unknown dataset: {name}")
