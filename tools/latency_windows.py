"""Time per step during which the GPU runs only latency kernels (a few workgroups each:
NMS, proposal decode / sort, target sampling, losses) — the serial stretches of the step
that leave the CUs idle even though a kernel is running.  From a rocprofv3 kernel trace.

usage: python tools/latency_windows.py run_kernel_trace.csv STEPS_IN_TRACE [LAST_STEPS]"""
import csv
import re
import sys
from collections import defaultdict

SMALL = re.compile(r"nms_|proposal|rocprim|trampoline|at_|pt_|rpn_loss|loss|detect|gather_sorted|"
                   r"fill|copyBuffer|reduce_kernel<|elementwise|softmax|argmax|index|cat_|scatter")


def main():
    fn, steps = sys.argv[1], int(sys.argv[2])
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ev = []
    for r in csv.DictReader(open(fn)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _ in ev)
    span = (t1 - t0) / steps
    lo = t1 - int(span * last)
    pts = []
    for s, e, n in ev:
        if e < lo:
            continue
        s = max(s, lo)
        small = bool(SMALL.search(n))
        pts.append((s, 1, small, n))
        pts.append((e, -1, small, n))
    pts.sort(key=lambda p: (p[0], p[1]))
    n_big = n_small = 0
    only_small = idle = 0
    who = defaultdict(int)
    active = defaultdict(int)
    prev = lo
    for t, d, small, n in pts:
        dt = t - prev
        if n_big == 0 and n_small > 0:
            only_small += dt
            for k, c in active.items():
                if c > 0:
                    who[re.sub(r"\(.*", "", k)[:70]] += dt
        elif n_big == 0 and n_small == 0:
            idle += dt
        prev = t
        if small:
            n_small += d
        else:
            n_big += d
        active[n] += d
    per = 1e-6 / last
    print(f"window {last} steps: only-latency-kernels {only_small * per:.3f} ms/step, idle {idle * per:.3f} ms/step")
    for k, v in sorted(who.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v * per:7.3f} ms/step  {k}")


if __name__ == "__main__":
    main()
