"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals over the span
of the last LAST_S seconds of the trace (the timed steps), and the longest idle gaps.

usage: python tools/gpu_busy.py run_kernel_trace.csv [LAST_S]"""
import csv
import sys


def main():
    fn = sys.argv[1]
    last = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    iv = []
    with open(fn) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    iv.sort()
    t_end = max(e for _, e, _ in iv)
    t0 = t_end - int(last * 1e9)
    iv = [x for x in iv if x[0] >= t0]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    prev_name = ""
    for s, e, n in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%), "
          f"{len(iv)} kernels, idle {sum(g for g, _, _ in gaps) / 1e6:.2f} ms in {len(gaps)} gaps")
    for g, a, b in sorted(gaps, reverse=True)[:12]:
        print(f"  gap {g / 1e3:8.1f} us after {a!r} before {b!r}")


if __name__ == "__main__":
    main()
