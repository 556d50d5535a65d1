#!/bin/bash
# parity tests, then an envs-per-wave sweep of the bench (each step time-boxed)
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for SC in robocup lunar; do for E in 1 2 4 8; do
  COTIX_ENVS_PER_WAVE=$E timeout -k 10 120 python bench.py --scenario $SC --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/prof/sweep_${SC}_EW$E.json 2>/dev/null || exit 1
  echo "$SC EW=$E $(python -c "import json;d=json.load(open('gpurun_out/prof/sweep_${SC}_EW$E.json'));print('%.4g'%d['value'], '%.4g'%d['roofline']['launch_ms'])")"
done; done
