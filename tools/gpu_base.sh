set -e
mkdir -p gpurun_out/r03d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d/gpu_tests.log 2>&1
tail -3 gpurun_out/r03d/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-others > gpurun_out/r03d/cfg4.json 2> gpurun_out/r03d/cfg4.err
tail -c 300 gpurun_out/r03d/cfg4.json
