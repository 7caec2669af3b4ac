#!/bin/bash
# Round-3 measurement set on the GPU box, each step under its own time limit, chained with &&:
#   new GPU tests, the default bench line (cfg4 + cfg5 block + CPU baselines), bench --workload cfg5
#   under torchrun with the nccl backend at world size 1, a rocprofv3 kernel-trace summary of the
#   default bench command, and PMC passes over the cfg5 launch shape and the cfg2 / cfg3 kernels.
#   tools/measure_r03.sh TAG [pytest selection...]
set -e
TAG=${1:-r03}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $OUT/gpu_tests.log 2>&1
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -c 600 $OUT/bench.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu --no-e2e --no-others > $OUT/bench_cfg5_nccl_w1.json 2> $OUT/bench_cfg5_nccl_w1.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-others --steps 5 > $OUT/trace.log 2>&1
bash tools/pmc_op.sh $OUT/pmc_cfg5 spm 25000000
bash tools/pmc_op.sh $OUT/pmc_cfg2 segment3 1000000 0
bash tools/pmc_op.sh $OUT/pmc_cfg3 analyze 1000000
echo "measure $TAG done"
