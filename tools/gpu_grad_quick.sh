set -o pipefail
O=gpurun_out/${TAG:-gq}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pytree.py -m gpu -x -q -k "grad or rollout or tape" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for sc in robocup box lunar; do timeout -k 10 200 python bench.py --mode grad --scenario $sc --extras off --cpu-baseline off > $O/g_$sc.json 2> $O/e_$sc.txt || { tail -3 $O/e_$sc.txt; exit 3; }; python -c "
import json; d=json.loads(open('$O/g_$sc.json').read().strip().split('\n')[-1]); c=d['config']; print('$sc', round(d['value']/1e6,1), round(c.get('fwd_ms'),4), round(c.get('bwd_ms'),4))"; done
