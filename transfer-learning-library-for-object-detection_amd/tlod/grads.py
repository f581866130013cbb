"""Persistent gradient storage: every trainable parameter's ``.grad`` lives in one flat
device buffer (the arena) at a fixed offset.

Why: the reference zeroes and re-accumulates ``.grad`` tensors every step
(``fasterRCNN.zero_grad()`` / ``optimizer.zero_grad()``, methods/DAF/DAF_train.py:386,404),
and ``set_to_none`` instead hands autograd a fresh allocation per step — either way the
gradient addresses move or cost a zero fill.  Here:

  * tlod's own autograd Functions (conv / linear weight and bias gradients) write their
    result straight into the parameter's arena slot (``claim``), and autograd adopts that
    tensor as ``.grad`` without a copy (AccumulateGrad steals a gradient nobody else holds);
  * a gradient produced elsewhere (the narrow nn.Linear heads) is copied into its slot by
    a post-accumulate hook, so after backward every ``.grad`` is a view of the arena;
  * the optimizer's per-chunk descriptor table (tlod.optim) therefore never changes and is
    uploaded once, and the data-parallel reducer (tlod.dist) all-reduces arena ranges in
    place.

Semantics stay those of ``zero_grad(set_to_none=True)``: a parameter that receives no
gradient in a step keeps ``.grad = None`` (torch.optim.SGD then skips it).  Under data
parallelism the reducer (tlod.dist) extends the arena by a tail of one float per parameter
(``tail``/``active``): the number of ranks that produced the parameter's gradient, summed by
the same all-reduce as the gradients, which the fused optimizer reads on the device.
"""
import torch

_ALIGN = 4  # floats: every slot starts on a 16-byte boundary (the float4 optimizer path)


def _pad(n):
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class GradArena:
    def __init__(self, params, order=None):
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("GradArena: no trainable parameters")
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or p.device != dev or not p.is_contiguous():
                raise TypeError("GradArena: contiguous float32 parameters on one device")
        self.params = params
        self.index = {p: i for i, p in enumerate(params)}
        self.gen = 0
        self.layout_gen = 0  # bumped by every layout(): keys tables built for a slot layout
        self._claimed = {}
        self._seen = {}
        self.n_seen = 0  # parameters whose gradient arrived (in its slot) this generation
        self.listeners = []
        self.tail_len = 0
        self.active = None  # per-parameter gradient-producer counts (tail view), DP only
        self.hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params]
        self.layout(order if order is not None else range(len(params)))

    def layout(self, order, tail=None):
        """(Re)assign slots in the given parameter order (indices into ``params``); existing
        gradients move along.  tail: floats reserved after the last slot (kept if None)."""
        order = [self.params[i] for i in order]
        assert len(order) == len(self.params) and len(set(order)) == len(order)
        if tail is not None:
            self.tail_len = _pad(int(tail))
        offs, off = {}, 0
        for p in order:
            offs[p] = off
            off += _pad(p.numel())
        self.tail_off = off
        flat = torch.zeros(off + self.tail_len, dtype=torch.float32,
                           device=self.params[0].device)
        old, old_active = getattr(self, "flat", None), getattr(self, "active", None)
        self.order, self.offset, self.flat = order, offs, flat
        self.layout_gen = getattr(self, "layout_gen", 0) + 1
        self.active = self.flat.narrow(0, off, len(self.params)) if self.tail_len else None
        if old_active is not None and self.active is not None:
            self.active.copy_(old_active)
        for p in order:
            p._tlod_grad_arena = self
            if old is not None and p.grad is not None:
                v = self.view(p)
                v.copy_(p.grad)
                p.grad = v

    def view(self, p):
        """A new view of p's slot (a fresh tensor object each call)."""
        return self.flat.narrow(0, self.offset[p], p.numel()).view_as(p)

    def span(self, p):
        return self.offset[p], _pad(p.numel())

    def claim(self, p):
        """The slot for a kernel to write p's gradient into, or None when p already holds a
        gradient (accumulation across backward calls) or the slot was handed out earlier in
        this step (p used twice in the graph: the engine sums the two contributions)."""
        if p.grad is not None or self._claimed.get(p) == self.gen:
            return None
        self._claimed[p] = self.gen
        return self.view(p)

    def zero_grad(self):
        self.gen += 1
        self.n_seen = 0
        for p in self.params:
            p.grad = None

    def _on_grad(self, p):
        g = p.grad
        off = self.offset[p]
        if g.data_ptr() != self.flat.data_ptr() + 4 * off:
            v = self.view(p)
            v.copy_(g)
            p.grad = v
        if self._seen.get(p) != self.gen:
            self._seen[p] = self.gen
            self.n_seen += 1
        for cb in self.listeners:
            cb(p)


def arena_of(p):
    return getattr(p, "_tlod_grad_arena", None)


def grad_out(p):
    """Output buffer for p's gradient: its arena slot when one is free, else None (the
    caller allocates)."""
    if p is None or not p.requires_grad:
        return None
    a = arena_of(p)
    return a.claim(p) if a is not None else None
