#!/bin/bash
# Development aid (GPU box): SPM parity tests, A/B default vs nested lattice, then blocks-per-CU caps.
set -e
bash tools/gpu_ab_spm.sh default nested
for b in 3 2; do AK_SPM_BPC=$b AB_ROWS=4000000 timeout -k 10 200 python -u tools/ab_ops.py spm | sed "s/default/bpc$b/" >> gpurun_out/ab.jsonl; done
tail -2 gpurun_out/ab.jsonl
