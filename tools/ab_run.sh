#!/bin/bash
# Development aid (GPU box): tools/ab_ops.py for each variant name given (and "default");
# AB_OPS="bpe spm" restricts the ops.
set -e
for v in "$@"; do
  if [ "$v" = default ]; then timeout -k 10 200 python -u tools/ab_ops.py $AB_OPS >> gpurun_out/ab.jsonl
  else AK_LIB_VARIANT=$v timeout -k 10 200 python -u tools/ab_ops.py $AB_OPS >> gpurun_out/ab.jsonl; fi
done
