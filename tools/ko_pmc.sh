#!/bin/bash
# Development aid (GPU box): per-pass counter costs of the BPE tile kernel. One rocprofv3 --pmc run
# over tools/prof_op.py bpe 4000000 for each build that returns after a pass (AK_KNOCKOUT 8..14,
# akshar_amd/_build.py build_variant) and for the full kernel; per-row differences = a pass's cost.
#   KO="ko8 ko9 ... default" PMC="SQ_INSTS_VMEM_RD SQ_INSTS_VALU ..." OUT=gpurun_out/kopmc tools/ko_pmc.sh
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/kopmc}
KO=${KO:-"ko8 ko9 ko10 ko11 ko12 ko13 ko14 default"}
PMC=${PMC:-"SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES"}
mkdir -p $OUT
for v in $KO; do
  if [ $v = default ]; then
    timeout -s KILL 120 rocprofv3 --pmc $PMC -d $OUT/$v -o $v --output-format csv -- python3 tools/prof_op.py bpe 4000000 1 1 > $OUT/$v.log 2>&1 || echo "$v failed"
  else
    AK_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $PMC -d $OUT/$v -o $v --output-format csv -- python3 tools/prof_op.py bpe 4000000 1 1 > $OUT/$v.log 2>&1 || echo "$v: the knocked-out build fails the output checks (counters still collected)"
  fi
  echo "$v done"
done
