#!/bin/bash
# The round's measurement set on the GPU box, each step under its own time limit, chained by set -e:
#   tests    the whole GPU suite                         smoke   __graft_entry__.smoke()
#   bench    the default bench line (cfg4 + cfg5 block + side configs + per-call latency + CPU baseline)
#   nccl     bench --workload cfg5 under torchrun (nccl, world 1)
#   trace    rocprofv3 kernel trace + stats of the cfg4 bench command
#   pmc      PMC passes over the cfg4 (10 M-row BPE) and cfg5 (25 M-row SPM) launch shapes (tools/pmc_op.sh)
#   pmcrows  PMC passes over the cfg2 (1 M Devanagari rows, segment) and cfg3 (1 M Hinglish, fused analyze) launches
#   fallback tools/fallback_realism.py
#   waves    tools/wave_split.py (the fallback waves' per-pass split, fuzz / alphabet sets)
#   tools/measure.sh TAG [STEP...]      (no steps: all of them, in this order)
set -e
TAG=${1:?tag}
shift || true
STEPS=${*:-tests smoke bench nccl trace pmc pmcrows fallback waves}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
           tail -1 $OUT/gpu_tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
           tail -1 $OUT/smoke.log ;;
    bench) timeout -k 10 700 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
           tail -c 300 $OUT/bench.json ;;
    nccl) timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
            --master-port 29513 bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu --no-e2e --no-others --no-single \
            > $OUT/bench_cfg5_nccl_w1.json 2> $OUT/bench_cfg5_nccl_w1.err ;;
    trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- \
             python3 bench.py --no-cpu --no-e2e --no-others --no-single --steps 5 > $OUT/trace.log 2>&1 ;;
    pmc) bash tools/pmc_op.sh $OUT/pmc_cfg4 bpe 10000000
         bash tools/pmc_op.sh $OUT/pmc_cfg5 spm 25000000 ;;
    pmcrows) bash tools/pmc_op.sh $OUT/pmc_cfg2 segment3 1000000 0
             bash tools/pmc_op.sh $OUT/pmc_cfg3 analyze 1000000 1 ;;
    fallback) timeout -k 10 400 python -u tools/fallback_realism.py > $OUT/fallback_realism.json 2> $OUT/fallback_realism.err ;;
    waves) timeout -k 10 300 python -u tools/wave_split.py > $OUT/wave_split.jsonl 2> $OUT/wave_split.err ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "measure $TAG done"
