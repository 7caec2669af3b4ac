#!/bin/bash
# Development aid (GPU box): SPM / BPE kernel rates under blocks-per-CU caps (AK_SPM_BPC / AK_TILE_BPC).
set -e
mkdir -p gpurun_out; rm -f gpurun_out/bpc.jsonl
for b in 0 3 2; do
  AK_SPM_BPC=$([ $b = 0 ] && echo 99 || echo $b) AB_ROWS=4000000 timeout -k 10 200 python -u tools/ab_ops.py spm | sed "s/\"default\"/\"spm_bpc$b\"/" >> gpurun_out/bpc.jsonl
done
for b in 0 1; do
  AK_TILE_BPC=$([ $b = 0 ] && echo 99 || echo $b) AB_ROWS=4000000 timeout -k 10 200 python -u tools/ab_ops.py bpe | sed "s/\"default\"/\"bpe_bpc$b\"/" >> gpurun_out/bpc.jsonl
done
cat gpurun_out/bpc.jsonl
