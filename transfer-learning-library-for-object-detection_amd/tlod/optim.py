"""Fused clip_gradient + SGD(momentum) on libtlod (tlod_sgd_clip_f32).

Same update as ``clip_gradient(model, 10.)`` (lib/model/utils/net_utils.py:38-49) followed
by ``torch.optim.SGD(params, momentum=0.9)`` with the reference's param groups
(methods/DAF/DAF_train.py:311-325: biases lr*(DOUBLE_BIAS+1) and no weight decay unless
BIAS_DECAY; weights lr and WEIGHT_DECAY) — three launches, no host wait: the gradients
live in the persistent arena (tlod.grads), so the descriptor table is built and uploaded
once per (arena layout, set of parameters with a gradient, learning rates).
"""
import os

import numpy as np
import torch

from . import _lib
from .grads import GradArena, arena_of

CHUNK = 65536
_DESC = np.dtype([("param", np.uint64), ("grad", np.uint64), ("buf", np.uint64),
                  ("count", np.int64), ("lr", np.float32), ("wd", np.float32),
                  ("active", np.uint64)])
assert _DESC.itemsize == 48  # sizeof(tlod_sgd_chunk), include/tlod.h


class FusedSGDClip:
    """param_groups: list of dicts {params, lr, weight_decay} (torch.optim.SGD layout)."""

    def __init__(self, param_groups, momentum=0.9, clip_norm=10.0):
        self.param_groups = [dict(g, params=[p for p in g["params"] if p.requires_grad])
                             for g in param_groups]
        self.momentum = float(momentum)
        self.clip_norm = float(clip_norm)
        self.params = [p for g in self.param_groups for p in g["params"]]
        for p in self.params:
            _lib.require_cuda(p)
        dev = self.params[0].device
        self.bufs = [torch.zeros_like(p) for p in self.params]
        n_chunks = sum((p.numel() + CHUNK - 1) // CHUNK for p in self.params)
        self.partials = torch.empty(n_chunks, dtype=torch.float32, device=dev)
        self.norm_scale = torch.zeros(2, dtype=torch.float32, device=dev)
        # gradient arena: reuse the one the parameters already belong to (e.g. the DP
        # reducer's), else create one in registration order
        a = arena_of(self.params[0])
        if a is None or any(arena_of(p) is not a for p in self.params):
            a = GradArena(self.params) if os.environ.get("TLOD_GRAD_ARENA", "1") != "0" else None
        self.arena = a
        # descriptor tables per gradient-pointer set; with the arena the key is stable and
        # the (blocking, tiny) upload happens on the first step only
        self._tables = {}
        self._key = None
        self._n = 0

    def zero_grad(self, set_to_none=True):
        if set_to_none and self.arena is not None:
            self.arena.zero_grad()
            return
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def _chunk_table(self):
        """Descriptor rows for every parameter that has a gradient (torch.optim.SGD skips
        the others entirely: no weight decay, no momentum update)."""
        grads = [p.grad for p in self.params]
        a = self.arena
        act = a.active if a is not None and a.active is not None else None
        key = tuple(0 if g is None else g.data_ptr() for g in grads) + \
            tuple(g["lr"] for g in self.param_groups) + (0 if act is None else act.data_ptr(),)
        hit = self._tables.get(key)
        if hit is not None:
            self._n = hit[1]
            return hit[0]
        rows = []
        idx = 0
        for g in self.param_groups:
            for p in g["params"]:
                gr, buf = p.grad, self.bufs[idx]
                if gr is None:
                    idx += 1
                    continue
                assert gr.is_contiguous() and p.is_contiguous()
                n = p.numel()
                # data parallel: skipped on the device when no rank produced the gradient
                ap = 0 if act is None else act.data_ptr() + 4 * a.index[p]
                for off in range(0, n, CHUNK):
                    rows.append((p.data_ptr() + 4 * off, gr.data_ptr() + 4 * off,
                                 buf.data_ptr() + 4 * off, min(CHUNK, n - off), g["lr"],
                                 g.get("weight_decay", 0.0), ap))
                idx += 1
        arr = np.array(rows, dtype=_DESC)
        table = torch.empty(arr.nbytes, dtype=torch.uint8, device=self.partials.device)
        if arr.nbytes:
            host = torch.empty(arr.nbytes, dtype=torch.uint8, pin_memory=True)
            host.numpy()[:] = arr.view(np.uint8)
            table.copy_(host)
        if len(self._tables) >= 8:
            self._tables.pop(next(iter(self._tables)))
        self._tables[key] = (table, len(rows))
        self._key, self._n = key, len(rows)
        return table

    @torch.no_grad()
    def step(self, grad_scale=1.0):
        """grad_scale: factor applied to every gradient as it is read (data parallel: 1/world
        of the all-reduced sums, tlod.dist.GradBucketReducer.grad_scale)."""
        table = self._chunk_table()
        if self._n == 0:
            return self.norm_scale[0]
        _lib.check(_lib.lib().tlod_sgd_clip_f32(
            _lib.ptr(table), self._n, float(grad_scale), self.momentum, self.clip_norm,
            _lib.ptr(self.partials), _lib.ptr(self.norm_scale), _lib.stream_of(self.partials)),
            "sgd_clip")
        return self.norm_scale[0]
