"""Data-parallel DAF-VGG16 training on the real model: two processes on cuda:0 with gloo
over device tensors (the one-GPU box stands in for two ranks; RCCL and gloo run the same
reducer code — SUM all-reduce, 1/world applied by the fused optimizer).

Checks after each of 2 steps of tlod.detector.train.train_step:
  * weights are bit-identical on both ranks;
  * they equal a single-process FusedSGDClip step on the two ranks' local gradients
    (captured before the all-reduce) summed and scaled by 1/2 — the DataParallel
    loss.mean() semantics of methods/DAF/DAF_train.py:341-342 / :397;
  * rank 1 runs a target image of a different size, so its forward takes the unbatched
    branch (tlod.da.daf) and finishes gradients in a different order than rank 0: the
    static bucket order must keep the collectives paired.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd")
H, W = 192, 320


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank, step, dev):
    from tlod.detector.train import SyntheticCityscapes
    b = list(SyntheticCityscapes(dev, H=H, W=W, G=4, pool=1, seed=50 + 10 * rank + step).next())
    if rank == 1:  # smaller target image: the unbatched forward branch
        t = SyntheticCityscapes(dev, H=H - 32, W=W, G=4, pool=1, seed=99 + step).next()
        b[5], b[6] = t[5], t[6]
    return tuple(b)


def _worker(rank, world, port, outdir, reserve=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    if reserve is not None:  # the nccl-only CU reserve, forced under gloo
        os.environ["TLOD_DIST_CU_RESERVE"] = str(reserve)
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    import tlod.dist as td
    from tlod.detector.train import build_model, make_optimizer, train_step
    from tlod.dist import GradBucketReducer
    calls = []
    real_set = td._set_cu_reserve
    td._set_cu_reserve = lambda n: (calls.append(int(n)), real_set(n))[1]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = build_model("daf", dev, "vgg16", seed=rank)  # rank 1's init is overwritten by rank 0's
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    opt = make_optimizer(m, 2e-3, clip=10.0)
    red = GradBucketReducer(m, bucket_mb=16.0)
    names = {p: k for k, p in m.named_parameters()}
    local = {}
    red.arena.listeners.insert(0, lambda p: local.__setitem__(names[p], p.grad.detach().clone()))
    rec = {"w0": {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}}
    for step in range(2):
        local.clear()
        train_step(m, opt, _batch(rank, step, dev), reducer=red)
        torch.cuda.synchronize()
        rec[f"g{step}"] = {k: v.cpu() for k, v in local.items()}
        rec[f"w{step + 1}"] = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    rec["reserve_calls"] = torch.tensor(calls, dtype=torch.int64)
    torch.save(rec, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("reserve", [None, 32])
def test_daf_vgg16_data_parallel_two_ranks(tmp_path, reserve):
    """reserve=32: TLOD_DIST_CU_RESERVE forced under gloo, so the reducer's reserve toggle
    (on at the first bucket's launch, off after finish(): tlod.dist) runs every backward of
    both steps, and each rank's conv / GEMM launches after fc6's bucket execute the plans for
    224 CUs that the 8-GPU RCCL run uses; the device-tensor broadcast of the first step's
    bucket order runs too (the arena lives on cuda:0)."""
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), reserve), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    want = [32, 0, 32, 0] if reserve else []
    assert r0["reserve_calls"].tolist() == want and r1["reserve_calls"].tolist() == want
    for step in (1, 2):
        for k in r0[f"w{step}"]:
            assert torch.equal(r0[f"w{step}"][k], r1[f"w{step}"][k]), (step, k)
    # single-process reference: rank 0's initial weights, FusedSGDClip on (g0 + g1) / 2
    sys.path.insert(0, PKG)
    from tlod.detector.train import build_model, make_optimizer
    dev = torch.device("cuda", 0)
    m = build_model("daf", dev, "vgg16", seed=0)
    m.load_state_dict({k: v.to(dev) for k, v in r0["w0"].items()}, strict=True)
    opt = make_optimizer(m, 2e-3, clip=10.0)
    for step in range(2):
        opt.zero_grad()
        n = 0
        for k, p in m.named_parameters():
            if k in r0[f"g{step}"]:
                assert k in r1[f"g{step}"], k
                p.grad = (r0[f"g{step}"][k].to(dev) + r1[f"g{step}"][k].to(dev)).contiguous()
                n += 1
        assert n == len(r0[f"g{step}"]) == len([p for p in m.parameters() if p.requires_grad])
        opt.step(grad_scale=0.5)
        torch.cuda.synchronize()
        for k, p in m.named_parameters():
            ref = p.detach().cpu()
            assert torch.equal(ref, r0[f"w{step + 1}"][k]), (step, k,
                                                              (ref - r0[f"w{step + 1}"][k]).abs().max())


def _worker_partial(rank, world, port, outdir):
    """Toy model on cuda:0, fused SGD: rank 1 never differentiates head2, and no rank
    differentiates `unused` (weight decay must not touch it)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from tlod.dist import GradBucketReducer
    from tlod.optim import FusedSGDClip
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(rank)
    m = torch.nn.ModuleDict({"trunk": torch.nn.Linear(32, 64), "head1": torch.nn.Linear(64, 48),
                             "head2": torch.nn.Linear(64, 7), "unused": torch.nn.Linear(3, 3)}).to(dev)
    opt = FusedSGDClip([{"params": list(m.parameters()), "lr": 0.1, "weight_decay": 1e-2}],
                       momentum=0.9, clip_norm=10.0)
    red = GradBucketReducer(m, bucket_mb=1e-4)
    w0 = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    for step in range(3):
        opt.zero_grad()
        red.zero_grad()
        g = torch.Generator().manual_seed(100 + 10 * rank + step)
        h = torch.relu(m["trunk"](torch.randn(16, 32, generator=g).to(dev)))
        loss = (m["head1"](h) ** 2).mean()
        if rank == 0:
            loss = loss + (m["head2"](h) ** 2).mean()
        loss.backward()
        red.finish()
        opt.step(grad_scale=red.grad_scale)
    torch.cuda.synchronize()
    torch.save({"w0": w0, "w": {k: v.detach().cpu().clone() for k, v in m.named_parameters()}},
               os.path.join(outdir, f"p{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_fused_sgd_partial_gradients_two_ranks(tmp_path):
    port = _free_port()
    mp.spawn(_worker_partial, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "p0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "p1.pt", weights_only=True)
    for k in r0["w"]:
        assert torch.equal(r0["w"][k], r1["w"][k]), k
    # head2 was updated (rank 0's gradient reached rank 1), unused was not touched at all
    assert not torch.equal(r0["w"]["head2.weight"], r0["w0"]["head2.weight"])
    assert torch.equal(r0["w"]["unused.weight"], r0["w0"]["unused.weight"])
    assert torch.equal(r0["w"]["unused.bias"], r0["w0"]["unused.bias"])


def _worker_cfg(rank, world, port, outdir, method, net):
    """BASELINE configs 3 and 5 (8-GPU DAF-R101 / ATF-R101) on two ranks: one step each."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from tlod.detector.train import build_model, make_optimizer, train_step
    from tlod.dist import GradBucketReducer
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = build_model(method, dev, net, seed=rank)  # rank 1's init is overwritten by rank 0's
    opt = make_optimizer(m, 2e-3, clip=10.0)
    red = GradBucketReducer(m, bucket_mb=16.0)
    w0 = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    loss = train_step(m, opt, _batch(rank, 0, dev), reducer=red)
    torch.cuda.synchronize()
    torch.save({"w0": w0, "loss": float(loss),
                "w": {k: v.detach().cpu().clone() for k, v in m.named_parameters()}},
               os.path.join(outdir, f"{method}{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("method,net", [("daf", "res101"), ("atf", "res101")])
def test_resnet101_configs_data_parallel_two_ranks(tmp_path, method, net):
    """Configs 3 / 5 run data-parallel: after one step on different images the two ranks'
    weights are bit-identical (the broadcast initial weights, the SUM all-reduce over the
    arena, the same fused update), finite, and moved."""
    port = _free_port()
    mp.spawn(_worker_cfg, args=(2, port, str(tmp_path), method, net), nprocs=2, join=True)
    r0 = torch.load(tmp_path / f"{method}0.pt", weights_only=True)
    r1 = torch.load(tmp_path / f"{method}1.pt", weights_only=True)
    moved = 0
    for k in r0["w"]:
        assert torch.equal(r0["w"][k], r1["w"][k]), k
        assert torch.isfinite(r0["w"][k]).all(), k
        moved += int(not torch.equal(r0["w"][k], r0["w0"][k]))
    assert moved > 0
    assert r0["loss"] == r0["loss"] and r1["loss"] == r1["loss"]  # not NaN
