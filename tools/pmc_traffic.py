"""Per-kernel HBM traffic per step from rocprofv3 PMC passes of bench.py.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR STEPS OUT.json

FETCH_SIZE / WRITE_SIZE are the L2 memory-side (fabric) request counters, in KiB.  Per
MI355X_MICROARCH.md (§HBM) FETCH_SIZE reports half the bytes of wide coalesced reads on
gfx950, so it is doubled (calibrated for these kernels in profiles/r01/pmc_calibration.md);
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted, so this is an upper bound on
HBM bytes.  STEPS = warmup + timed steps of the profiled run (every launch is counted).
"""
import csv
import glob
import json
import re
import sys


def kernel_key(name):
    """'void tlod::conv_fwd_bs_kernel<1, 8, ...>(float const*, ...)' -> 'conv_fwd_bs_kernel'."""
    name = name.replace("(anonymous namespace)::", "")
    base = re.split(r"[<(]", name, maxsplit=1)[0]
    return base.split("::")[-1].replace("void ", "").strip()[:80]


def total(path, counter):
    by = {}
    files = glob.glob(path + "/**/*counter_collection.csv", recursive=True)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                k = kernel_key(r["Kernel_Name"])
                by[k] = by.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return by


def main():
    fdir, wdir, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch, write = total(fdir, "FETCH_SIZE"), total(wdir, "WRITE_SIZE")
    keys = sorted(set(fetch) | set(write))
    per = {k: (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) / steps for k in keys}
    per = dict(sorted(((k, round(v)) for k, v in per.items() if v >= 1e5), key=lambda kv: -kv[1]))
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (separate runs) over "
                     "python3 bench.py --steps 10 --warmup 3 --cpu-baseline-steps 0",
           "steps_profiled": steps,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> B",
           "bytes_per_step_by_kernel": per, "bytes_per_step": round(sum(per.values()))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()
