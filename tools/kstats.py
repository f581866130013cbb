"""Summarise a rocprofv3 run_kernel_stats.csv per training step: ms/step per kernel
(grouped by kernel name without arguments), sorted.  usage: python tools/kstats.py CSV STEPS [N]"""
import csv
import re
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    agg = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Name"])
        a = agg.setdefault(k, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"])
    tot = sum(v[1] for v in agg.values())
    print(f"total kernel time {tot / 1e6 / steps:.3f} ms/step over {steps} steps")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / 1e6 / steps:8.3f} ms/step {c / steps:7.1f} calls/step {t / c / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
