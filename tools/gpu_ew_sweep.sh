#!/bin/bash
# envs-per-wave sweep of the bench (--envs-per-wave: a kernel variant, same bits)
set -o pipefail
mkdir -p gpurun_out/ew
for E in 1 2 4 8; do for SC in robocup lunar; do
  [ "$SC$E" = lunar8 ] && continue  # LunarLander's tile does not fit the LDS at 8 envs per wave
  timeout -k 10 120 python bench.py --envs-per-wave $E --scenario $SC --steps 20 --warmup 3 --cpu-baseline off --extras off > gpurun_out/ew/b_${SC}_$E.json 2> gpurun_out/ew/e.err || { tail gpurun_out/ew/e.err; exit 1; }
  echo "$SC EW=$E $(python -c "import json;d=json.load(open('gpurun_out/ew/b_${SC}_$E.json'));print('%.4g'%d['value'], 'launch_ms %.4g'%d['roofline']['launch_ms'])")"
done; done
