#!/bin/bash
# Issue-time breakdown of a tile kernel (GPU box): cycles each instruction class is issued,
# instruction fetch, and the kernel's cycles.   tools/pmc_issue.sh OUTDIR OP ROWS
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/issue}; OP=${2:-bpe}; ROWS=${3:-4000000}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/$OP" -o issue --output-format csv -- python3 tools/prof_op.py "$OP" "$ROWS" 1 1 > "$OUT/$OP.log" 2>&1
echo "issue $OP done"
