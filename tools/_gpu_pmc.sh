set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
A="$*"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc1 -o run -- python3 tools/conv_kernels_once.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/pmc2 -o run -- python3 tools/conv_kernels_once.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3 -o run -- python3 tools/conv_kernels_once.py $A > /dev/null 2>&1 || true
ls gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
