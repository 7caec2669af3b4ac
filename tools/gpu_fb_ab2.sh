#!/bin/bash
# Development aid (GPU box): encode parity tests, then tools/gpu_fb_ab.sh over the variants given.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "spm or bpe or synthetic or long or empty or tie or golden" > gpurun_out/enc_tests.log 2>&1
tail -2 gpurun_out/enc_tests.log
bash tools/gpu_fb_ab.sh "$@"
