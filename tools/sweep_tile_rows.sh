set -e
for R in 16 4; do
  AK_TILE_ROWS=$R timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-others > gpurun_out/sweep_cfg4_R$R.json 2>/dev/null
  AK_TILE_ROWS=$R timeout -k 10 200 python -u bench.py --workload cfg5 --rows 20000000 --steps 3 --warmup 1 --no-cpu --no-e2e --no-others > gpurun_out/sweep_cfg5_R$R.json 2>/dev/null
done
