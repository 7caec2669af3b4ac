#!/bin/bash
# Development aid (GPU box): encode parity tests, then the SPM kernel rate at full occupancy and
# capped to 4 blocks per CU (AK_SPM_BPC).
set -e
mkdir -p gpurun_out; rm -f gpurun_out/occ.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py tests/test_spm_rebase.py -m gpu -x -q --timeout 300 --timeout-method thread -k "spm or synthetic or long or empty or tie or golden or cli or rebase" > gpurun_out/enc_tests.log 2>&1
tail -1 gpurun_out/enc_tests.log
for r in 1 2; do for b in 99 4; do
  AK_SPM_BPC=$b AB_ROWS=4000000 timeout -k 10 200 python -u tools/ab_ops.py spm | sed "s/\"default\"/\"spm_bpc$b\"/" >> gpurun_out/occ.jsonl
done; done
cat gpurun_out/occ.jsonl
