"""Per-kernel PMC summary of rocprofv3 --pmc csv passes (usage: pmc_summary.py DIR...)."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for d in sys.argv[1:]:
    with open(d + "/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0][-60:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
for k, v in agg.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:28s} {v[c] / max(1, cnt[k][c]):16.1f} per dispatch")
    w = v.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
            if c in v:
                print(f"   {c + '/WAVE':28s} {v[c] / w:8.3f}")
