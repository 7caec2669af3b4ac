#!/bin/bash
# Round profile (run on the GPU box): kernel trace + stats of the default bench, then separate PMC
# passes (HBM bytes, SQ instruction mix) over one cfg4-size tile-path encode.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
ROWS=${2:-10000000}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bench" -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 > "$OUT/bench_stdout.log" 2> "$OUT/bench_stderr.log"
pmc() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 tools/prof_op.py bpe "$ROWS" 1 1 > "$OUT/$name.log" 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
echo profile done
