#!/bin/bash
# compare builds of the library (compiler-flag experiments): for each .so in
# LIBS, the parity traces + ragged tests, then the RoboCup / LunarLander bench.
# Every GPU step time-boxed; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/libcmp; mkdir -p $O
for L in $LIBS; do
  n=$(basename $L .so)
  COTIX_AMD_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "trace or ragged or 4096" > $O/pytest_$n.log 2>&1
  rc=$?; echo "$n pytest rc=$rc $(tail -1 $O/pytest_$n.log)"; [ $rc -eq 0 ] || exit $rc
  for SC in robocup lunar; do
    COTIX_AMD_LIB=$PWD/$L timeout -k 10 120 python bench.py --scenario $SC --steps 20 --warmup 3 --cpu-baseline off > $O/bench_${n}_$SC.json 2> $O/bench_${n}_$SC.err || { tail $O/bench_${n}_$SC.err; exit 1; }
    echo "$n $SC $(python -c "import json;d=json.load(open('$O/bench_${n}_$SC.json'));print('%.4g'%d['value'], 'launch_ms %.4g'%d['roofline']['launch_ms'])")"
  done
done
