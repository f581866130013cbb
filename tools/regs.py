"""Per-kernel VGPR / spill summary of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/regs.py FILE.hip [-DNAME=V ...]   (run from csrc/)"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
       "-I../../include", "-c", sys.argv[1], "-o", "/tmp/regs.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
name = None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        name, row = v, {}
    else:
        row[k] = v
        if k == "VGPRs Spill":
            short = re.sub(r"^_ZN4tlod(12_GLOBAL__N_1)?\d+", "", name)[:70]
            print(f"{row.get('VGPRs', '?'):>4} vgpr  spill {v:>4}  occ {row.get('Occupancy [waves/SIMD]', '?')}  {short}")
