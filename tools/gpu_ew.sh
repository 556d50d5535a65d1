#!/bin/bash
# envs-per-wave sweep of the step kernel (both scenarios)
set -o pipefail
mkdir -p gpurun_out/ew
for sc in robocup lunar; do for ew in 1 2 4; do
  COTIX_ENVS_PER_WAVE=$ew timeout -k 10 120 python bench.py --scenario $sc --cpu-baseline off --steps 10 --warmup 2 > gpurun_out/ew/${sc}_$ew.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ew/${sc}_$ew.json'));print('$sc EW=$ew', round(d['value']/1e6,1), 'M/s', round(d['roofline']['launch_ms'],3),'ms')"
done; done
