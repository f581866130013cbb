"""Data parallelism for the DAF step: one process per GPU, RCCL all-reduce over xGMI.

Replaces the reference's single-process ``nn.DataParallel`` (methods/DAF/DAF_train.py:
341-342), which at ``--bs 1`` never runs more than one replica and reduces gradients to
GPU 0 through the host thread.  Here:

  * parameters are broadcast from rank 0 once at start;
  * large parameters (>= ``direct_numel`` elements: the conv and fc weights, 98% of the
    568 MB) are all-reduced in place as single messages from their post-accumulate-grad
    hook, on the gradient tensor autograd produced (set_to_none: no zero fill, no
    accumulate-add, no copy into a bucket);
  * the small ones (biases, the narrow heads) have ``.grad`` views into flat buckets so
    they travel in few messages; a hook counts ready parameters per bucket and launches
    the bucket's async all-reduce when it is complete;
  * every all-reduce is async (ReduceOp.AVG on RCCL — the DataParallel loss.mean()
    semantics) and overlaps the rest of the backward (fc6/fc7 are ready first: the heads
    backprop before the backbone);
  * ``finish()`` waits for the outstanding buckets before clip_gradient / SGD, which
    then run on identical gradients on every rank (no extra collective for the norm).

Bucket sizing targets point-to-point xGMI rings: few, large messages (default 64 MB).
"""
import os

import torch
import torch.distributed as dist


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


class GradBucketReducer:
    def __init__(self, model, bucket_mb=64.0, group=None, direct_numel=1 << 20):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.direct = {p for p in self.params if p.numel() >= direct_numel}
        self.direct_work = []
        backend = dist.get_backend(group)
        self.avg = backend == "nccl"
        # broadcast initial weights (and buffers) from rank 0
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0, group=group)
        # buckets in reverse registration order (~ gradient readiness order)
        cap = int(bucket_mb * 1024 * 1024 / 4)
        buckets, cur, cur_n = [], [], 0
        for p in reversed([q for q in self.params if q not in self.direct]):
            if cur and cur_n + p.numel() > cap:
                buckets.append(cur)
                cur, cur_n = [], 0
            cur.append(p)
            cur_n += p.numel()
        if cur:
            buckets.append(cur)
        self.buckets = []
        self.bucket_of = {}
        for bi, ps in enumerate(buckets):
            n = sum(p.numel() for p in ps)
            flat = torch.zeros(n, dtype=ps[0].dtype, device=ps[0].device)
            off = 0
            for p in ps:
                p.grad = flat[off:off + p.numel()].view_as(p)
                self.bucket_of[p] = bi
                off += p.numel()
            self.buckets.append({"flat": flat, "params": ps, "ready": 0, "work": None})
        self.hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def zero_grad(self):
        for b in self.buckets:
            b["flat"].zero_()
            b["ready"] = 0
            b["work"] = None
        for p in self.direct:
            p.grad = None
        self.direct_work = []

    def _launch(self, b):
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        b["work"] = dist.all_reduce(b["flat"], op=op, group=self.group, async_op=True)

    def _on_grad(self, p):
        if p in self.direct:
            op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
            self.direct_work.append(
                (p, dist.all_reduce(p.grad, op=op, group=self.group, async_op=True)))
            return
        b = self.buckets[self.bucket_of[p]]
        b["ready"] += 1
        if b["ready"] == len(b["params"]):
            self._launch(b)

    def finish(self):
        for b in self.buckets:
            if b["work"] is None:
                self._launch(b)
        for b in self.buckets:
            b["work"].wait()
            if not self.avg:
                b["flat"].div_(self.world)
            b["work"] = None
            b["ready"] = 0
        for p, w in self.direct_work:
            w.wait()
            if not self.avg:
                p.grad.div_(self.world)
        if len(self.direct_work) != len(self.direct):
            raise RuntimeError("GradBucketReducer: a large parameter received no gradient this "
                               "step (every rank must all-reduce the same tensors)")
        self.direct_work = []
        # small grads must still alias the flat buffers (zero them with reducer.zero_grad())
        for p in self.params:
            assert p.grad is not None
