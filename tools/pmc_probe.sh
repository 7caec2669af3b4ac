#!/bin/bash
# Development aid (GPU box): list the PMC counters, then memory-pipe counters for the SPM tile kernel
# of the default library and of a variant (AK_LIB_VARIANT).   tools/pmc_probe.sh VARIANT
set -e
export TMPDIR=/tmp
OUT=gpurun_out/probe
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "^[ ]*[A-Z][A-Z0-9_]*" $OUT/avail.txt | sort -u | grep -E "^ *(TA_|TD_|TCP_|TCC_HIT|TCC_MISS|TCC_REQ|GRBM_GUI|SQ_INST_CYCLES|SQ_BUSY_CU|SQ_LDS|SQ_INSTS_V)" > $OUT/names.txt || true
run() {  # name variant counters...
    local name=$1 var=$2; shift 2
    AK_LIB_VARIANT=$var timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- python3 tools/prof_op.py spm 2000000 1 1 > "$OUT/$name.log" 2>&1
}
for v in "" "$@"; do
  tag=${v:-default}
  run ta_$tag "$v" TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum GRBM_GUI_ACTIVE
  run td_$tag "$v" TD_TD_BUSY_sum TD_SPI_STALL_sum GRBM_COUNT
  run tcp_$tag "$v" TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
done
echo probe done
