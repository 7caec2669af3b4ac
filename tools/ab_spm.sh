#!/bin/bash
# SentencePiece A/B on the GPU box (development aid): the GPU tests named by TESTS, then kernel MB/s
# of tools/ab_ops.py spm (AB_ROWS rows) for each environment setting and library variant, twice.
set -e
TAG=${TAG:?tag}
mkdir -p gpurun_out/$TAG
if [ -n "${TESTS-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/$TAG/gpu_tests.log 2>&1
  tail -1 gpurun_out/$TAG/gpu_tests.log
fi
for rep in 1 2; do
  for e in ${AB_ENVS:-X=1}; do
    for v in ${AB_VARIANTS:-default}; do
      if [ "$v" = default ]; then env -u AK_LIB_VARIANT $e AB_TAG="$e" AB_DETAIL=1 timeout -k 10 300 python -u tools/ab_ops.py spm >> gpurun_out/$TAG/ab.jsonl
      else env $e AK_LIB_VARIANT=$v AB_TAG="$e" AB_DETAIL=1 timeout -k 10 300 python -u tools/ab_ops.py spm >> gpurun_out/$TAG/ab.jsonl; fi
    done
  done
done
cat gpurun_out/$TAG/ab.jsonl
