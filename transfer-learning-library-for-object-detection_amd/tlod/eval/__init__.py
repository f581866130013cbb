"""Test-time detection and PASCAL VOC evaluation (methods/*/*_test.py, lib/datasets/voc_eval.py)."""
