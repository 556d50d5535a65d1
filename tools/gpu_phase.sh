#!/bin/bash
# per-phase cost of the step kernel: time with phases skipped (COTIX_DEBUG_SKIP
# bits: T=1 B=2 C=4 D=8 A-keys=16 E=32); results are garbage, timing only
set -o pipefail
mkdir -p gpurun_out/phase
for sc in robocup lunar; do
for skip in 0 1 2 4 8 16 32 12 63; do
  COTIX_DEBUG_SKIP=$skip timeout -k 10 120 python bench.py --scenario $sc --cpu-baseline off --steps 10 --warmup 2 > gpurun_out/phase/${sc}_skip$skip.json 2>/dev/null || { echo "fail $sc $skip"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/phase/${sc}_skip$skip.json'));print('$sc skip=$skip', round(d['roofline']['launch_ms'],4))"
done
done
