#!/bin/bash
# PMC passes over one tile-path BPE encode of 1 M synthetic Hinglish rows (run on the GPU box).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
run() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 tools/prof_op.py bpe 1000000 1 1 > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run sq2 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc done
