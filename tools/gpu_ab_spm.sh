#!/bin/bash
# Development aid (GPU box): SPM parity tests on the default build, then an A/B of variants.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "spm or synthetic or long or empty or ties or tie" > gpurun_out/spm_tests.log 2>&1
tail -2 gpurun_out/spm_tests.log
export AB_ROWS=${AB_ROWS:-4000000} AB_OPS=${AB_OPS:-spm}
rm -f gpurun_out/ab.jsonl
bash tools/ab_run.sh "$@"
bash tools/ab_run.sh "$@"
cat gpurun_out/ab.jsonl
