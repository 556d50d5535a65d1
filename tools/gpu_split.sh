#!/bin/bash
# split tape backward (cxk::run_backward_split): the gradient parity subset,
# then an A/B of the config-5 benches against the one-wave tape backward
# (COTIX_SPLIT_BWD=0), alternated.  Every GPU step time-boxed; stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-split}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pytree.py -m gpu -x -v -k "grad or rollout or tape" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 0 1; do
    for sc in robocup box; do
      COTIX_SPLIT_BWD=$sp timeout -k 10 200 python bench.py --mode grad --scenario $sc --extras off --cpu-baseline off > $O/g_${sc}_$sp.json 2> $O/e_${sc}_$sp.txt || { tail -3 $O/e_${sc}_$sp.txt; exit 3; }
      python -c "
import json; d=json.loads(open('$O/g_${sc}_$sp.json').read().strip().split('\n')[-1]); c=d['config']; print('split=$sp', '$sc', round(d['value']/1e6,1), 'fwd', round(c.get('fwd_ms'),4), 'bwd', round(c.get('bwd_ms'),4))"
    done
  done
done
