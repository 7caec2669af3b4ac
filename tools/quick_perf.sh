#!/bin/bash
# Quick perf check on the GPU box: cfg4 and a 20 M-row cfg5, kernel-resident, no side legs.
set -e
TAG=${1:-q}
timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-others > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err
timeout -k 10 200 python -u bench.py --workload cfg5 --rows 20000000 --steps 3 --warmup 1 --no-cpu --no-e2e --no-others > gpurun_out/${TAG}_cfg5.json 2> gpurun_out/${TAG}_cfg5.err
