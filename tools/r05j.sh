set -e
TAG=${TAG:-r05x}
mkdir -p gpurun_out/$TAG
if [ -n "$FIRST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$FIRST" > gpurun_out/$TAG/gpu_first.log 2>&1
  tail -1 gpurun_out/$TAG/gpu_first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
tail -1 gpurun_out/$TAG/gpu_tests.log
timeout -k 10 500 python -u tools/fallback_realism.py > gpurun_out/$TAG/fallback_realism.json 2> gpurun_out/$TAG/fallback_realism.err
if [ -n "$AB_VARIANTS" ]; then TAG=$TAG AB_ROWS=4000000 timeout -k 10 600 bash tools/ab_spm.sh; fi
