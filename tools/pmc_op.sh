#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over one op of tools/prof_op.py, on the GPU box:
#   tools/pmc_op.sh OUTDIR OP ROWS [KIND: 0 Devanagari, 1 Hinglish (default)]
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
OP=${2:-spm}
ROWS=${3:-1000000}
KIND=${4:-1}
mkdir -p "$OUT"
pmc() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 tools/prof_op.py "$OP" "$ROWS" "$KIND" 1 > "$OUT/$name.log" 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
pmc sq2 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
pmc mem TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
pmc tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- python3 tools/prof_op.py "$OP" "$ROWS" "$KIND" 3 > "$OUT/trace.log" 2>&1
echo "pmc $OP done"
