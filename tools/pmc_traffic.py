"""Per-step HBM traffic of the conv kernels from rocprofv3 PMC passes of bench.py.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR STEPS CALLS_PER_STEP OUT.json

FETCH_SIZE / WRITE_SIZE are the L2 memory-side (fabric) request counters, in KiB.  Per
MI355X_MICROARCH.md (§HBM) FETCH_SIZE reports half the bytes of wide coalesced reads on
gfx950, so it is doubled; WRITE_SIZE is taken as is.  Infinity-Cache hits are counted, so
this is an upper bound on HBM bytes.  STEPS = warmup + timed steps of the profiled run.
"""
import csv
import json
import sys

CONV = ("conv_fwd_kernel", "conv_wgrad_kernel", "conv_fwd_bs_kernel", "conv_wgrad_bs_kernel",
        "fwd_tail_reduce_kernel", "slab_reduce_kernel", "relu_bwd_bias_kernel", "pack_fwd_kernel",
        "pack_dgrad_kernel", "pack_bs_kernel")


def total(path, counter):
    by = {}
    with open(path + "/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            key = next((k for k in CONV if k + "<" in name or k + "(" in name), None)
            if key:
                by[key] = by.get(key, 0.0) + float(r["Counter_Value"]) * 1024.0
    return by


def main():
    fdir, wdir, steps, calls, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    fetch, write = total(fdir, "FETCH_SIZE"), total(wdir, "WRITE_SIZE")
    per_step = {k: (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) / steps for k in CONV}
    tot = sum(per_step.values())
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py",
           "steps_profiled": steps, "conv_calls_per_step": calls,
           "bytes_per_step_by_kernel": {k: round(v) for k, v in per_step.items() if v},
           "bytes_per_step": round(tot), "bytes_per_call": round(tot / calls),
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> B"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
