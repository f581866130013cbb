"""Faster R-CNN detector pieces on the tlod kernels: backbone, RPN head, losses, train step."""
