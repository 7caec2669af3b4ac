set -e
# SentencePiece word pool A/B (4 M rows): kernel ms per class, pass split, with the redo kernel
TAG=${TAG:-r05f}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "spm" > gpurun_out/$TAG/gpu_tests.log 2>&1
tail -1 gpurun_out/$TAG/gpu_tests.log
for e in "AK_SPM_POOL=0" "AK_SPM_POOL_MIN=2" "AK_SPM_POOL_MIN=4" "AK_SPM_POOL=0" "AK_SPM_POOL_MIN=2" "AK_SPM_POOL_MIN=4"; do
  env $e AB_TAG="$e" AB_DETAIL=1 AB_ROWS=4000000 timeout -k 10 300 python -u tools/ab_ops.py spm >> gpurun_out/$TAG/ab.jsonl
done
for e in "AK_SPM_POOL=0" "AK_SPM_POOL_MIN=2"; do
  env $e AB_TAG="$e" timeout -k 10 300 python -u tools/pass_split.py spm 4000000 1 >> gpurun_out/$TAG/passes.jsonl
done
cat gpurun_out/$TAG/ab.jsonl gpurun_out/$TAG/passes.jsonl
