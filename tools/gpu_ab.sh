#!/bin/bash
# Development aid (GPU box): encode parity tests on the default build, then A/B of library variants
# (tools/ab_ops.py, AB_OPS / AB_ROWS), each twice.   tools/gpu_ab.sh VARIANT...
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "spm or bpe or synthetic or long or empty or tie" > gpurun_out/enc_tests.log 2>&1
tail -2 gpurun_out/enc_tests.log
export AB_ROWS=${AB_ROWS:-4000000} AB_OPS=${AB_OPS:-"spm bpe"}
rm -f gpurun_out/ab.jsonl
bash tools/ab_run.sh default "$@"
bash tools/ab_run.sh default "$@"
cat gpurun_out/ab.jsonl
if [ -n "$AB_FALLBACK" ]; then
  timeout -k 10 300 python -u tools/fallback_realism.py > gpurun_out/fallback_realism.json 2> gpurun_out/fallback_realism.err
  tail -c 400 gpurun_out/fallback_realism.json
fi
