"""Fused clip_gradient + SGD(momentum) on libtlod (tlod_sgd_clip_f32).

Same update as ``clip_gradient(model, 10.)`` (lib/model/utils/net_utils.py:38-49) followed
by ``torch.optim.SGD(params, momentum=0.9)`` with the reference's param groups
(methods/DAF/DAF_train.py:311-325: biases lr*(DOUBLE_BIAS+1) and no weight decay unless
BIAS_DECAY; weights lr and WEIGHT_DECAY) — three launches, no host wait: the gradients
live in the persistent arena (tlod.grads), so the descriptor table is built and uploaded
once per (arena layout, set of parameters with a gradient, learning rates).

3x3 conv weights are updated by tiles that also write their split-bf16 packs (the conv
kernels' operand layouts, tlod_sgd_clip_pack_f32): the optimizer marks them as owned
(`_tlod_pack_owner`), tlod.conv.pack_bs then caches their packs, and the next forward and
backward use the packs this step wrote instead of re-packing every weight.  TLOD_SGD_PACK=0
turns that off (every trainable 3x3 weight re-packed per use, as before; such an optimizer
also takes back the ownership an earlier one claimed, and drops the cached packs of weights a
later one claimed after each of its plain updates, so no pack outlives its weight).  Weight
writes outside these optimizers that bypass the version counter (``p.data.*_()``, a direct
tlod_sgd_clip_f32 call) must call tlod.conv.weights_updated(), as the data-parallel broadcast
does.
"""
import os

import numpy as np
import torch

from . import _lib
from . import conv as _conv
from .grads import GradArena, arena_of

CHUNK = 65536
_DESC = np.dtype([("param", np.uint64), ("grad", np.uint64), ("buf", np.uint64),
                  ("count", np.int64), ("lr", np.float32), ("wd", np.float32),
                  ("active", np.uint64)])
assert _DESC.itemsize == 48  # sizeof(tlod_sgd_chunk), include/tlod.h
_TILE = np.dtype([("param", np.uint64), ("grad", np.uint64), ("buf", np.uint64),
                  ("active", np.uint64), ("pack_fwd", np.uint64), ("pack_dgrad", np.uint64),
                  ("pack_dgrad_scaled", np.uint64), ("scale", np.uint64), ("lr", np.float32),
                  ("wd", np.float32), ("cout", np.int32), ("cin", np.int32), ("o0", np.int32),
                  ("i0", np.int32), ("reserved", np.int32, 2)])
assert _TILE.itemsize == 96  # sizeof(tlod_sgd_pack_tile), include/tlod.h
TILE = 32  # channels per tile side (optim.hip kPT)


def _packs_of(p):
    """(fwd pack, dgrad pack, scaled dgrad pack, its scale) the fused update can keep
    current, or None when the weight has none yet."""
    packs = getattr(p, "_tlod_packs", None)
    if not packs:
        return None
    pf = pd = pds = sc = None
    for (dgrad, skey), (_, pk, scale) in packs.items():
        if skey is None:
            if dgrad:
                pd = pk
            else:
                pf = pk
        elif dgrad:
            pds, sc = pk, scale
    return (pf, pd, pds, sc) if (pf is not None or pd is not None or pds is not None) else None


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
        self.fused_packs = os.environ.get("TLOD_SGD_PACK", "1") != "0"
        for p in self.params:
            if p.dim() == 4 and tuple(p.shape[2:]) == (3, 3):
                if self.fused_packs:
                    p._tlod_pack_owner = True
                elif getattr(p, "_tlod_pack_owner", False):
                    # this optimizer's plain update would leave an earlier owner's cached
                    # packs stale: the weight goes back to a repack per use (round-5 advisor)
                    p._tlod_pack_owner = False
                    p._tlod_packs = {}
                    _conv.PACK_GEN[0] += 1
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
        self.table_builds = 0  # descriptor-table (re)builds: each is a blocking upload

    def zero_grad(self, set_to_none=True):
        if set_to_none and self.arena is not None:
            self.arena.zero_grad()
            return
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def _upload(self, arr):
        table = torch.empty(max(arr.nbytes, 1), dtype=torch.uint8, device=self.partials.device)
        if arr.nbytes:
            host = torch.empty(arr.nbytes, dtype=torch.uint8, pin_memory=True)
            host.numpy()[:] = arr.view(np.uint8)
            table.copy_(host)
        return table

    def _chunk_table(self, fast=True):
        """Descriptor rows for every parameter that has a gradient (torch.optim.SGD skips
        the others entirely: no weight decay, no momentum update): (chunk table, tile table,
        rows updated by chunks, rows, tiles).  The 3x3 weights with packs get tiles; their
        chunk rows (negative counts) only enter the gradient norm."""
        a = self.arena
        act = a.active if a is not None and a.active is not None else None
        tail = tuple(g["lr"] for g in self.param_groups) + \
            (0 if act is None else act.data_ptr(), _conv.PACK_GEN[0] if self.fused_packs else 0)
        # fast key: with the arena, a step in which every parameter's gradient arrived has
        # every gradient in its fixed slot (GradArena._on_grad), so the table depends only on
        # the arena, the learning rates and the packs (no per-parameter host work: ~0.6 ms
        # of Python per ResNet101 step, the GPU idling at the end of the backward)
        if fast and a is not None and a.n_seen == len(a.params) and \
                all(arena_of(p) is a for p in self._fast_ok()):
            # (the layout generation, not the buffer address: a relayout's new buffer may
            # land where an earlier one was freed)
            key = ("all", id(a), a.layout_gen) + tail
        else:
            key = tuple(0 if p.grad is None else p.grad.data_ptr() for p in self.params) + tail
        hit = self._tables.get(key)
        if hit is not None:
            return hit
        self.table_builds += 1
        rows, tiles, keep = [], [], []
        idx = 0
        for g in self.param_groups:
            for p in g["params"]:
                gr, buf = p.grad, self.bufs[idx]
                idx += 1
                if gr is None:
                    continue
                assert gr.is_contiguous() and p.is_contiguous()
                n = p.numel()
                lr, wd = g["lr"], g.get("weight_decay", 0.0)
                # data parallel: skipped on the device when no rank produced the gradient
                ap = 0 if act is None else act.data_ptr() + 4 * a.index[p]
                packs = _packs_of(p) if self.fused_packs and getattr(p, "_tlod_pack_owner",
                                                                     False) else None
                # every parameter's chunk rows in parameter order (the norm's summation order
                # does not depend on TLOD_SGD_PACK); a negative count marks a norm-only row,
                # whose elements the pack tiles update
                sign = 1 if packs is None else -1
                for off in range(0, n, CHUNK):
                    rows.append((p.data_ptr() + 4 * off, gr.data_ptr() + 4 * off,
                                 buf.data_ptr() + 4 * off, sign * min(CHUNK, n - off), lr, wd, ap))
                if packs is None:
                    continue
                keep.append(packs)  # the table holds their pointers
                pf, pd, pds, sc = (0 if t is None else t.data_ptr() for t in packs)
                cout, cin = p.shape[0], p.shape[1]
                for o0 in range(0, cout, TILE):
                    for i0 in range(0, cin, TILE):
                        tiles.append((p.data_ptr(), gr.data_ptr(), buf.data_ptr(), ap, pf, pd,
                                      pds, sc, lr, wd, cout, cin, o0, i0, (0, 0)))
        chunks = self._upload(np.array(rows, dtype=_DESC))
        tile_t = self._upload(np.array(tiles, dtype=_TILE))
        if len(self._tables) >= 8:
            self._tables.pop(next(iter(self._tables)))
        hit = (chunks, tile_t, len(rows), len(rows), len(tiles), keep)
        self._tables[key] = hit
        return hit

    def _fast_ok(self):
        """() once the optimizer's parameters are known to be exactly the arena's (checked
        once), else the parameters (the fast key then requires each to be in the arena)."""
        if getattr(self, "_fast_checked", None) is None:
            a = self.arena
            self._fast_checked = (a is not None and set(a.params) == set(self.params))
        return () if self._fast_checked else self.params

    @torch.no_grad()
    def step(self, grad_scale=1.0):
        """grad_scale: factor applied to every gradient as it is read (data parallel: 1/world
        of the all-reduced sums, tlod.dist.GradBucketReducer.grad_scale)."""
        # the fast key needs a zero_grad (a new arena generation) since the last step
        gen = self.arena.gen if self.arena is not None else None
        fast = gen is not None and gen != getattr(self, "_last_gen", None)
        self._last_gen = gen
        chunks, tiles, n_update, n, n_tiles, _ = self._chunk_table(fast)
        if n == 0:
            return self.norm_scale[0]
        _lib.check(_lib.lib().tlod_sgd_clip_pack_f32(
            _lib.ptr(chunks), n, n_update, _lib.ptr(tiles), n_tiles, float(grad_scale),
            self.momentum, self.clip_norm, _lib.ptr(self.partials), _lib.ptr(self.norm_scale),
            _lib.stream_of(self.partials)), "sgd_clip")
        if not self.fused_packs:
            # the plain update writes weights without a version bump: packs cached for a
            # weight that a pack-writing optimizer claimed after this one was built are stale
            for p in self.params:
                if getattr(p, "_tlod_pack_owner", False) and getattr(p, "_tlod_packs", None):
                    p._tlod_packs = {}
                    _conv.PACK_GEN[0] += 1
        return self.norm_scale[0]
