# Effective clock, MFMA busy and LDS counters of the conv kernels (conv3_3 microbench).
set -e
O=gpurun_out/clk
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for m in 0 2; do
rm -rf $O/p1_$m $O/p2_$m
TLOD_CONV_WS=$m timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1_$m -o run -- python3 tools/bench_conv.py --math bf16x6 > $O/p1_$m.json 2> $O/p1_$m.err
TLOD_CONV_WS=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $O/p2_$m -o run -- python3 tools/bench_conv.py --math bf16x6 > $O/p2_$m.json 2> $O/p2_$m.err
echo "=== WS=$m"
python3 tools/pmc_summary.py $O/p1_$m $O/p2_$m | grep -A14 "conv_fwd_bs"
python3 - $O/p1_$m <<'PY'
import csv,sys
from collections import defaultdict
d=defaultdict(list)
for r in csv.DictReader(open(sys.argv[1]+'/run_kernel_trace.csv')):
    d[r['Kernel_Name'].split('(')[0][-40:]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in d.items(): print(f"{k:42s} n={len(v)} avg_us={sum(v)/len(v):.1f}")
PY
done
