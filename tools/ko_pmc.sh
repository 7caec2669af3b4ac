#!/bin/bash
# per-pass VMEM / VALU / SALU counts via knockout variants (development aid)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/kopmc
mkdir -p $OUT
for v in ko9 ko10 ko11 ko12 ko13 ko14; do
  if [ $v = default ]; then
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -d $OUT/$v -o $v --output-format csv -- python3 tools/prof_op.py bpe 4000000 1 1 > $OUT/$v.log 2>&1 || echo "$v: the knocked-out build fails the output checks (counters still collected)"
  else
    AK_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -d $OUT/$v -o $v --output-format csv -- python3 tools/prof_op.py bpe 4000000 1 1 > $OUT/$v.log 2>&1 || echo "$v: the knocked-out build fails the output checks (counters still collected)"
  fi
  echo "$v done"
done
