#!/bin/bash
# Round-3 final measurement set on the GPU box, each step under its own time limit, chained by set -e:
#   the whole GPU suite, the default bench line (cfg4 + cfg5 block + CPU baselines), bench --workload
#   cfg5 under torchrun (nccl, world 1), a rocprofv3 kernel-trace summary of the bench command, PMC
#   passes over the cfg4 (10 M-row BPE) and cfg5 (25 M-row SPM) launch shapes, fallback realism.
#   tools/measure_r03f.sh TAG
set -e
TAG=${1:-r03f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -c 300 $OUT/bench.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu --no-e2e --no-others > $OUT/bench_cfg5_nccl_w1.json 2> $OUT/bench_cfg5_nccl_w1.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-others --steps 5 > $OUT/trace.log 2>&1
bash tools/pmc_op.sh $OUT/pmc_cfg4 bpe 10000000
bash tools/pmc_op.sh $OUT/pmc_cfg5 spm 25000000
timeout -k 10 400 python -u tools/fallback_realism.py > $OUT/fallback_realism.json 2> $OUT/fallback_realism.err
echo "measure $TAG done"
