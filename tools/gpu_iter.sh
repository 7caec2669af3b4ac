#!/bin/bash
# One GPU iteration (development aid, GPU box): the GPU suite (or a -k subset), optional A/B of
# environment settings and of library variants (akshar_amd/_build.py build_variant, selected by
# AK_LIB_VARIANT) on tools/ab_ops.py, and a short bench. Results under gpurun_out/$TAG.
#   TAG=x TESTS=all|none|"<pytest -k expression>" AB_ENVS="AK_PTC=0;" AB_VARIANTS="default v1" AB_OPS="bpe"
#   AB_ROWS=4000000 BENCH="--no-cpu" tools/gpu_iter.sh
set -e
TAG=${TAG:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
T=${TESTS-all}
if [ "$T" = all ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
elif [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$T" > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
fi
if [ -n "${AB_ENVS-}" ]; then
  IFS=';' read -ra ENVS <<< "$AB_ENVS"
  for rep in 1 2; do
    for e in "${ENVS[@]}"; do
      env $e AB_TAG="$e" timeout -k 10 300 python -u tools/ab_ops.py ${AB_OPS-bpe} >> $OUT/ab.jsonl
    done
  done
  cat $OUT/ab.jsonl
fi
if [ -n "${AB_VARIANTS-}" ]; then
  for rep in 1 2; do
    for v in $AB_VARIANTS; do
      if [ "$v" = default ]; then timeout -k 10 300 python -u tools/ab_ops.py ${AB_OPS-bpe} >> $OUT/ab.jsonl
      else AK_LIB_VARIANT=$v timeout -k 10 300 python -u tools/ab_ops.py ${AB_OPS-bpe} >> $OUT/ab.jsonl; fi
    done
  done
  cat $OUT/ab.jsonl
fi
if [ "${BENCH-none}" != "none" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $OUT/bench.json 2> $OUT/bench.err
  tail -c 300 $OUT/bench.json
fi
