"""Writes small synthetic datasets in the VOC layout the reference reads
(lib/datasets/pascal_voc.py:91-131, 218-271): JPEGImages/*.jpg, Annotations/*.xml,
ImageSets/Main/<set>.txt.  No real dataset is available offline; these drive the data
layer, the source-only / DAF training paths and the VOC evaluation end to end.  Source
domain images are named ``source_*`` (lib/DAF/minibatch.py:34-38 keys need_backprop on it).
"""
import os
import xml.etree.ElementTree as ET

import numpy as np
from PIL import Image


def _xml(index, H, W, objects):
    root = ET.Element("annotation")
    ET.SubElement(root, "filename").text = index + ".jpg"
    size = ET.SubElement(root, "size")
    for k, v in (("width", W), ("height", H), ("depth", 3)):
        ET.SubElement(size, k).text = str(v)
    for (name, x1, y1, x2, y2, difficult) in objects:
        o = ET.SubElement(root, "object")
        ET.SubElement(o, "name").text = name
        ET.SubElement(o, "pose").text = "Unspecified"
        ET.SubElement(o, "truncated").text = "0"
        ET.SubElement(o, "difficult").text = str(int(difficult))
        b = ET.SubElement(o, "bndbox")
        for k, v in (("xmin", x1), ("ymin", y1), ("xmax", x2), ("ymax", y2)):
            ET.SubElement(b, k).text = str(int(v))
    return ET.ElementTree(root)


def random_objects(rng, H, W, classes, n):
    """n boxes in 1-based VOC pixel coordinates, 32..min(400, side) wide, in the image."""
    objs = []
    for _ in range(n):
        w = int(rng.integers(32, min(400, W - 2)))
        h = int(rng.integers(32, min(400, H - 2)))
        x1 = int(rng.integers(1, W - w))
        y1 = int(rng.integers(1, H - h))
        objs.append((classes[int(rng.integers(1, len(classes)))], x1, y1, x1 + w, y1 + h, 0))
    return objs


def write_voc(devkit, images, year="2007", image_set="trainval", quality=95):
    """images: list of (index, uint8 HxWx3 RGB array, objects) with objects
    [(class_name, xmin, ymin, xmax, ymax, difficult)] in 1-based VOC coordinates."""
    d = os.path.join(devkit, "VOC" + year)
    for sub in ("JPEGImages", "Annotations", os.path.join("ImageSets", "Main")):
        os.makedirs(os.path.join(d, sub), exist_ok=True)
    for index, img, objects in images:
        Image.fromarray(img).save(os.path.join(d, "JPEGImages", index + ".jpg"), quality=quality)
        _xml(index, img.shape[0], img.shape[1], objects).write(
            os.path.join(d, "Annotations", index + ".xml"))
    with open(os.path.join(d, "ImageSets", "Main", image_set + ".txt"), "a") as f:
        for index, _, _ in images:
            f.write(index + "\n")
    return devkit


def synthetic_voc(devkit, sizes, classes, seed=0, n_objects=6, prefix="source_", year="2007",
                  image_set="trainval"):
    """One image per (H, W) in ``sizes``: uniform random pixels and ``n_objects`` boxes."""
    rng = np.random.default_rng(seed)
    images = []
    for i, (H, W) in enumerate(sizes):
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        images.append((f"{prefix}{i:06d}", img, random_objects(rng, H, W, classes, n_objects)))
    return write_voc(devkit, images, year, image_set)
