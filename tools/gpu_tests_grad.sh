#!/bin/bash
# GPU check of a build: the -m gpu suite, then the config-5 figures (grad
# RoboCup, box world, LunarLander settled).  Every GPU step time-boxed; the
# chain stops at the first failure.  TAG names gpurun_out/$TAG.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-check}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for sc in robocup box lunar; do
  timeout -k 10 300 python bench.py --mode grad --scenario $sc --steps 5 --cpu-baseline off > $O/grad_$sc.json 2> $O/grad_$sc.err
  rc=$?; echo "grad $sc rc=$rc"; [ $rc -eq 0 ] || { tail $O/grad_$sc.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('$O/grad_$sc.json')); c=d['config']; print('$sc', round(d['value']/1e6,1), 'M fwd', round(c['fwd_ms'],3), 'bwd', round(c['bwd_ms'],3))"
done
