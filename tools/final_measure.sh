#!/bin/bash
# Round-end measurement set on the GPU box (each step under its own time limit, chained):
#   GPU tests, the default bench line (cfg4, with the CPU baseline / end-to-end / other configs),
#   the cfg5 bench line, a rocprofv3 kernel-trace summary of the cfg4 bench command, the PMC
#   passes over one cfg4-size tile-kernel launch, and a 2-rank gloo rehearsal of the N > 1 path.
#   tools/final_measure.sh TAG
set -e
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu --no-e2e --no-others > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-others --steps 5 > $OUT/trace.log 2>&1
bash tools/pmc_op.sh $OUT/pmc_cfg4 bpe 10000000
AK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --rows 2000000 --no-cpu --no-e2e --no-others > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err
AK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload cfg5 --steps 3 --warmup 1 --rows 4000000 --no-cpu --no-e2e --no-others > $OUT/bench_n2_gloo_cfg5.json 2> $OUT/bench_n2_gloo_cfg5.err
echo "final measure $TAG done"
