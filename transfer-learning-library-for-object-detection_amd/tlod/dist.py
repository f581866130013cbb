"""Data parallelism for the DAF step: one process per GPU, RCCL all-reduce over xGMI.

Replaces the reference's single-process ``nn.DataParallel`` (methods/DAF/DAF_train.py:
341-342), which at ``--bs 1`` never runs more than one replica and reduces gradients to
GPU 0 through the host thread.  Here:

  * parameters and buffers are broadcast from rank 0 once at start;
  * every trainable gradient lives in the persistent arena (tlod.grads.GradArena), cut
    into contiguous buckets (default 32 MB; a larger tensor — fc6's 411 MB — is a bucket
    of its own); the all-reduce runs in place on the arena, no bucket copies;
  * the buckets form ONE static list, identical on every rank, and are launched strictly
    in that order: a gradient hook only marks its parameter ready, then the longest ready
    prefix of the list is launched (async).  Ranks whose graphs finish gradients in a
    different order (e.g. one rank batches source + target through one backbone pass and
    another does not, tlod.da.daf) still issue the same collectives in the same order;
  * the list order is the reverse parameter registration order for the first step; at the
    end of the first step rank 0's observed gradient-ready order is broadcast and the
    arena is re-laid out in it (once), so later steps launch each bucket as soon as its
    last gradient lands;
  * the reduction is SUM on every backend (the gloo tests run the production path); the
    1/world of DataParallel's ``loss.mean()`` semantics is applied by the fused optimizer
    as it reads the gradients (``grad_scale``), or by ``finish(scale=True)`` in place;
  * ``finish()`` waits for every bucket before clip_gradient / SGD, which then run on
    identical gradients on every rank (no extra collective for the norm).
"""
import os

import torch
import torch.distributed as dist

from .conv import weights_updated
from .grads import GradArena, arena_of


def init_from_env(backend=None):
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torch.distributed.run)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            device_id=torch.device("cuda", local) if backend == "nccl" else None)
    return rank, world


def _set_cu_reserve(n):
    from . import _lib
    _lib.check(_lib.lib().tlod_set_cu_reserve(int(n)), "set_cu_reserve")


class GradBucketReducer:
    def __init__(self, model, bucket_mb=32.0, group=None, relayout=True, arena=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.grad_scale = 1.0 / self.world
        params = [p for p in model.parameters() if p.requires_grad]
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, dist.get_global_rank(group, 0) if group else 0,
                               group=group)
        weights_updated()  # written through .data: no version bump
        if arena is None:
            arena = arena_of(params[0]) if params else None
            if arena is None or set(arena.params) != set(params):
                arena = GradArena(params)
        # first-step bucket order: reverse registration (the heads' gradients are ready
        # first), also when the arena was created by the optimizer in forward order; the
        # tail holds one gradient-producer count per parameter (see finish())
        n = len(arena.params)
        arena.layout(range(n - 1, -1, -1), tail=n)
        self.arena = arena
        self.cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        self.relayout_pending = relayout
        self.seen = []  # rank-local gradient-ready order of this step (parameter indices)
        # CUs the kernels' round planners leave free while the step's all-reduces run beside
        # the backward (tlod_set_cu_reserve): RCCL's kernels hold a few CUs, and a grid
        # planned for exactly one round of all 256 would run a second round for the few
        # workgroups left over.  With a 32-workgroup HBM-streaming stand-in launched at fc6's
        # gradient, the DAF-VGG16 backward took +2.8 ms with no reserve and +0.8 ms with 32
        # (profiles/r05/overlap_contention.json); a reserve costs ~8% on the
        # kernels it covers when nothing competes, so it is on only while collectives are in
        # flight, and only for RCCL (gloo reduces on the host).
        backend = dist.get_backend(group)
        self.cu_reserve = int(os.environ.get("TLOD_DIST_CU_RESERVE",
                                             "32" if backend == "nccl" else "0"))
        self._reserve_on = False
        self._build_buckets()
        arena.listeners.append(self._on_grad)

    # ------------------------------------------------------------------ layout
    def _build_buckets(self):
        a = self.arena
        self.buckets, self.bucket_of = [], {}
        cur, start, end = [], None, None
        for p in a.order:
            off, n = a.span(p)
            if cur and (off + n - start) > self.cap:
                self.buckets.append({"params": cur, "lo": start, "hi": end})
                cur = []
            if not cur:
                start = off
            cur.append(p)
            end = off + n
        if cur:
            self.buckets.append({"params": cur, "lo": start, "hi": end})
        # the producer-count tail rides on the last bucket (contiguous with it), which
        # therefore launches from finish() once every rank knows its own set
        self.buckets[-1]["hi"] = a.tail_off + a.tail_len
        for bi, b in enumerate(self.buckets):
            for p in b["params"]:
                self.bucket_of[p] = bi
        self._reset()

    def _reset(self):
        # a step abandoned before finish() (an exception in backward, zero_grad) must not
        # leave every later launch planned for fewer CUs (round-5 advisor)
        self._clear_reserve()
        for b in self.buckets:
            b["ready"], b["work"] = 0, None
        self.next = 0  # first bucket of the static list not yet launched
        self.marked = set()
        self.seen = []

    # ------------------------------------------------------------------ step
    def zero_grad(self):
        self.arena.zero_grad()
        self._reset()

    def _flat(self, b):
        return self.arena.flat[b["lo"]:b["hi"]]

    def _launch_ready_prefix(self):
        while self.next < len(self.buckets):
            b = self.buckets[self.next]
            if b["ready"] != len(b["params"]) + (self.next == len(self.buckets) - 1):
                return
            if self.next == 0 and self.cu_reserve:
                _set_cu_reserve(self.cu_reserve)
                self._reserve_on = True
            b["work"] = dist.all_reduce(self._flat(b), op=dist.ReduceOp.SUM, group=self.group,
                                        async_op=True)
            self.next += 1

    def _on_grad(self, p):
        if p in self.marked:
            raise RuntimeError("GradBucketReducer: a parameter received its gradient twice in "
                               "one step (gradient accumulation needs zero_grad() between "
                               "steps)")
        self.marked.add(p)
        self.seen.append(self.arena.index[p])
        b = self.buckets[self.bucket_of[p]]
        b["ready"] += 1
        self._launch_ready_prefix()

    def finish(self, scale=False):
        """Launch what is left (in list order) and wait.

        A parameter this rank gave no gradient contributes zeros.  Every rank writes 1 into
        the parameter's producer-count slot (arena tail) when it did produce the gradient,
        and the count is summed with the last bucket, so all ranks agree on which
        parameters were used anywhere (DataParallel's Broadcast backward sums the replicas'
        gradients, treating a missing one as zeros):
          * used on some rank: .grad is the reduced slot on every rank (also where this rank
            produced none — without this, that rank would skip its update and the weights
            and clip norm would diverge silently);
          * used on no rank: the fused optimizer skips it on the device (count 0), as
            torch.optim.SGD skips a None gradient; with scale=True (host optimizers) the
            counts are read back and such gradients are set to None.
        scale=True: also divide the gradients by the world size here (for optimizers that
        take no grad_scale)."""
        a = self.arena
        unmarked = [p for p in a.params if p not in self.marked]
        for b in self.buckets[self.next:]:
            for p in b["params"]:
                if p not in self.marked:
                    a.view(p).zero_()
            b["ready"] = len(b["params"])
        if unmarked:
            m = torch.ones(len(a.params), dtype=torch.float32)
            for p in unmarked:
                m[a.index[p]] = 0.0
            a.active.copy_(m)
        else:
            a.active.fill_(1.0)
        self.buckets[-1]["ready"] += 1
        self._launch_ready_prefix()
        for b in self.buckets:
            b["work"].wait()
        self._clear_reserve()
        for p in unmarked:
            p.grad = a.view(p)
        seen = self.seen
        if self.relayout_pending:
            self._relayout(seen)
        if scale:
            a.flat[:a.tail_off].mul_(self.grad_scale)
            used = (a.active > 0).tolist()
            for p in a.params:
                if not used[a.index[p]]:
                    p.grad = None
        self._reset()
        return seen

    def _clear_reserve(self):
        if getattr(self, "_reserve_on", False):
            _set_cu_reserve(0)
            self._reserve_on = False

    def _relayout(self, seen):
        """Adopt rank 0's gradient-ready order of the first step (broadcast, so every rank
        builds the same bucket list)."""
        self.relayout_pending = False
        n = len(self.arena.params)
        order = seen + [i for i in range(n) if i not in set(seen)]
        # the arena's device (RCCL; gloo broadcasts device tensors through the host), a CPU
        # tensor for a CPU arena
        dev = self.arena.flat.device
        t = torch.tensor(order, dtype=torch.int64, device=dev)
        dist.broadcast(t, dist.get_global_rank(self.group, 0) if self.group else 0,
                       group=self.group)
        self.arena.layout(t.cpu().tolist())  # moves the gradients and the counts along
        self._build_buckets()
