#!/bin/bash
# round-6 two-wave forms: the full GPU suite (split tape backward and key
# helper are the defaults), then A/Bs against their one-wave forms
# (COTIX_SPLIT_BWD=0, COTIX_KEY_HELPER=0), alternated.  Every GPU step
# time-boxed; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6d}; mkdir -p $O
[ "${TESTS:-1}" = 1 ] && { timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc; }
for rep in 1 2; do
  for kh in 0 1; do
    timeout -k 10 200 python bench.py --key-helper $kh --scenario robocup --extras off --cpu-baseline off > $O/s_$kh.json 2> $O/e_$kh.txt || { tail -3 $O/e_$kh.txt; exit 3; }
    python -c "
import json; d=json.loads(open('$O/s_$kh.json').read().strip().split('\n')[-1]); print('helper=$kh', round(d['value']/1e6,1), round(d['ms_per_step'],4))"
  done
  for sp in 0 1; do
    for sc in robocup box; do
      timeout -k 10 200 python bench.py --split-bwd $sp --mode grad --scenario $sc --extras off --cpu-baseline off > $O/g_${sc}_$sp.json 2> $O/ge_${sc}_$sp.txt || { tail -3 $O/ge_${sc}_$sp.txt; exit 4; }
      python -c "
import json; d=json.loads(open('$O/g_${sc}_$sp.json').read().strip().split('\n')[-1]); c=d['config']; print('split=$sp', '$sc', round(d['value']/1e6,1), 'fwd', round(c.get('fwd_ms'),4), 'bwd', round(c.get('bwd_ms'),4))"
    done
  done
done
