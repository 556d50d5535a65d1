#!/bin/bash
# A/B of two library builds on one box (perf tooling): LIBS="a.so b.so",
# ARGS = bench arguments; alternates the builds REP times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for r in $(seq 1 ${REP:-2}); do
  for L in $LIBS; do
    timeout -k 10 200 python bench.py --lib parallax_amd/_lib/$L $ARGS --cpu-baseline off --extras off > $O/ab_${L}_$r.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_${L}_$r.json'));print('$L', round(d['value']/1e6,1), round(d['roofline']['launch_ms'],4))"
  done
done
