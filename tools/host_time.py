"""Host-side (enqueue) time per training step vs the GPU step time: if the host needs about
as long to issue a step as the GPU needs to run it, the GPU idles between launches.
usage: python tools/host_time.py [steps] [net] [method]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "transfer-learning-library-for-object-detection_amd"))
import torch  # noqa: E402

from tlod.detector.train import (SyntheticCityscapes, build_model, make_optimizer,  # noqa: E402
                                 train_step)

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
net = sys.argv[2] if len(sys.argv) > 2 else "vgg16"
method = sys.argv[3] if len(sys.argv) > 3 else "daf"
dev = torch.device("cuda", 0)
model = build_model(method, dev, net)
opt = make_optimizer(model, 2e-3, clip=10.0)
data = SyntheticCityscapes(dev, H=600, W=1200, seed=1)
for _ in range(5):
    train_step(model, opt, data.next())
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for _ in range(steps):
    a = time.perf_counter()
    train_step(model, opt, data.next())
    host.append(time.perf_counter() - a)
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"host enqueue ms/step mean {1e3 * sum(host) / steps:.2f} (min {1e3 * min(host):.2f}, "
      f"max {1e3 * max(host):.2f}); wall ms/step {1e3 * t_all / steps:.2f}; "
      f"enqueue finished at {1e3 * t_enq / steps:.2f} ms/step")

print(f"optimizer descriptor-table builds: {getattr(opt, 'table_builds', '?')} over "
      f"{steps + 5} steps")
if os.environ.get("DIAG_STEP"):
    # host time of each phase of train_step, and whether the host waited on the GPU there
    from tlod.detector import train as _tr
    ph = {"fwd": [], "bwd": [], "opt": []}
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        out = model(*data.next())
        loss = model.total_loss(out, 0.1)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        opt.step()
        t3 = time.perf_counter()
        ph["fwd"].append(t1 - t0)
        ph["bwd"].append(t2 - t1)
        ph["opt"].append(t3 - t2)
    torch.cuda.synchronize()
    for k, v in ph.items():
        print(f"host {k}: mean {1e3 * sum(v) / len(v):.2f} ms (max {1e3 * max(v):.2f})")
    print(f"table builds now {opt.table_builds}")
if os.environ.get("HOST_PROFILE"):
    import cProfile
    import pstats
    if os.environ.get("HOST_PROFILE") == "bwd":
        # run the backward on this thread so cProfile sees the Python backward functions
        torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        train_step(model, opt, data.next())
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats(os.environ.get("HOST_SORT", "tottime")).print_stats(45)
