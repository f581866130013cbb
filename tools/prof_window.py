"""Summarise a rocprofv3 rocpd database over the timed steps of bench.py: GPU busy vs
idle time per step and the kernels by total time (usage: prof_window.py DB [warmup])."""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
ends = [r[2] for r in rows if "sgd_update_kernel" in r[0]]
t0, t1 = ends[warm - 1], ends[-1]
steps = len(ends) - warm
win = [r for r in rows if r[1] >= t0 and r[2] <= t1]
busy, cur_s, cur_e = 0, None, None
for _, s, e in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print(f"steps {steps}: wall {span / steps / 1e6:.3f} ms/step, GPU busy {busy / steps / 1e6:.3f}, "
      f"idle {(span - busy) / steps / 1e6:.3f}, kernels/step {len(win) / steps:.0f}")
by = defaultdict(lambda: [0, 0])
for n, s, e in win:
    k = n.split("(")[0][:90]
    by[k][0] += e - s
    by[k][1] += 1
for k, (t, n) in sorted(by.items(), key=lambda kv: -kv[1][0])[:45]:
    print(f"{t / steps / 1e3:9.1f} us/step {n / steps:6.1f}x  {k}")
