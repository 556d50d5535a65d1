#!/bin/bash
# key-window helper wave (cxk::KeyHelper): the full GPU suite, then an A/B of
# the RoboCup step bench against step_kernel alone (COTIX_KEY_HELPER=0),
# alternated, and the config-5 benches.  Every GPU step time-boxed; stops at
# the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-keyhelp}; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2 3; do
  for kh in 0 1; do
    COTIX_KEY_HELPER=$kh timeout -k 10 200 python bench.py --scenario robocup --extras off --cpu-baseline off > $O/s_$kh.json 2> $O/e_$kh.txt || { tail -3 $O/e_$kh.txt; exit 3; }
    python -c "
import json; d=json.loads(open('$O/s_$kh.json').read().strip().split('\n')[-1]); print('helper=$kh', round(d['value']/1e6,1), round(d['ms_per_step'],4))"
  done
done
for sc in robocup box; do
  timeout -k 10 200 python bench.py --mode grad --scenario $sc --extras off --cpu-baseline off > $O/g_$sc.json 2> $O/ge_$sc.txt || { tail -3 $O/ge_$sc.txt; exit 4; }
  python -c "
import json; d=json.loads(open('$O/g_$sc.json').read().strip().split('\n')[-1]); c=d['config']; print('grad', '$sc', round(d['value']/1e6,1), 'fwd', round(c.get('fwd_ms'),4), 'bwd', round(c.get('bwd_ms'),4))"
done
