#!/bin/bash
# Development aid (GPU box): tools/fallback_realism.py for the default library and each variant.
set -e
mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then timeout -k 10 300 python -u tools/fallback_realism.py > gpurun_out/fb_$v.json 2> gpurun_out/fb_$v.err
  else AK_LIB_VARIANT=$v timeout -k 10 300 python -u tools/fallback_realism.py > gpurun_out/fb_$v.json 2> gpurun_out/fb_$v.err; fi
  tail -c 200 gpurun_out/fb_$v.json
done
