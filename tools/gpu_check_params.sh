#!/bin/bash
# GPU check of a working tree: every -m gpu test, smoke, and the headline bench
# in both PRNG layouts (no extras); each GPU step time-boxed, stop at the first
# failure.  TAG names gpurun_out/$TAG.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-check}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/smoke.log; exit $rc; }
for L in legacy partitionable; do
  timeout -k 10 300 python bench.py --extras off --cpu-baseline off --prng-layout $L > $O/bench_$L.json 2> $O/bench_$L.err
  rc=$?; echo "bench $L rc=$rc"; cut -c1-300 $O/bench_$L.json; [ $rc -eq 0 ] || { tail $O/bench_$L.err; exit $rc; }
done
