"""Per-kernel averages of a rocprofv3 --pmc pass: duration, counters, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md DVFS), grouped by kernel and grid.

usage: python tools/pmc_kernel.py PMC_DIR [NAME_SUBSTRING]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def key(name):
    name = name.replace("(anonymous namespace)::", "")
    base = re.split(r"[(]", name, maxsplit=1)[0]
    return base.replace("void ", "").replace("tlod::", "").strip()[:70]


def main():
    d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    disp = {}
    for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                if sub not in r["Kernel_Name"]:
                    continue
                e = disp.setdefault(r["Dispatch_Id"], {"k": key(r["Kernel_Name"]), "grid": r["Grid_Size"],
                                                        "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = defaultdict(list)
    for e in disp.values():
        agg[(e["k"], e["grid"])].append(e)
    for (k, g), es in sorted(agg.items(), key=lambda kv: -sum(x["ns"] for x in kv[1])):
        n = len(es)
        ns = sum(x["ns"] for x in es) / n
        cnt = {c: sum(x.get(c, 0.0) for x in es) / n for c in es[0] if c not in ("k", "grid", "ns")}
        line = f"{k} grid={g} n={n} us={ns / 1e3:.1f}"
        if "GRBM_GUI_ACTIVE" in cnt:
            line += f" clock_GHz={cnt['GRBM_GUI_ACTIVE'] / 8 / ns:.3f}"
        line += " " + " ".join(f"{c}={v:.4g}" for c, v in sorted(cnt.items()))
        print(line)


if __name__ == "__main__":
    main()
