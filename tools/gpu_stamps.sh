#!/bin/bash
# K = 1 per-wave timeline (tools/k1_stamps.py) at K = 1 and 64, time-boxed
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stamps}; mkdir -p $O
timeout -k 10 120 python tools/k1_stamps.py > $O/k1.json 2> $O/k1.err || { tail -5 $O/k1.err; exit 3; }
timeout -k 10 120 python tools/k1_stamps.py --steps 64 --launches 50 > $O/k64.json 2> $O/k64.err || { tail -5 $O/k64.err; exit 4; }
cat $O/k1.json $O/k64.json
timeout -k 10 120 python tools/k1_loop.py > $O/k1_loop.json 2> $O/k1_loop.err || { tail -5 $O/k1_loop.err; exit 5; }
cat $O/k1_loop.json
if [ -n "$PYTEST" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; exit $rc
fi
