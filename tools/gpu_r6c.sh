#!/bin/bash
# full GPU suite, then the config-5 benches (fwd / bwd ms)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log; grep -E "FAILED|Error" $O/pytest_gpu.log | head -5
[ $rc -eq 0 ] || exit $rc
for sc in robocup box lunar; do timeout -k 10 200 python bench.py --mode grad --scenario $sc --extras off --cpu-baseline off > $O/g_$sc.json 2> $O/e_$sc.txt || { tail -3 $O/e_$sc.txt; exit 3; }; python -c "
import json; d=json.loads(open('$O/g_$sc.json').read().strip().split('\n')[-1]); c=d['config']; print('$sc', round(d['value']/1e6,1), round(c.get('fwd_ms'),4), round(c.get('bwd_ms'),4))"; done
if [ -n "$PHASES" ]; then
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
for sc in $PHASES; do
  timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario $sc --launches 3 > $O/phase_grad_$sc.json 2> $O/phase_grad_$sc.err || { tail -5 $O/phase_grad_$sc.err; exit 4; }
  python -c "
import json; d=json.load(open('$O/phase_grad_$sc.json'))
for k in ('forward','backward'):
    p=d[k]; print('$sc', k, round(p['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in p['phases'].items() if b['cycles_per_wave_step']>40})"
done
fi
if [ -n "$STEPPHASES" ]; then
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
for spec in $STEPPHASES; do  # name:args
  n=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
  timeout -k 10 200 python tools/phase_prof.py --lib $L $args > $O/phase_$n.json 2> $O/phase_$n.err || { tail -5 $O/phase_$n.err; exit 5; }
  python -c "
import json; p=json.load(open('$O/phase_$n.json'))
print('$n', round(p['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in p['phases'].items() if b['cycles_per_wave_step']>40})"
done
fi
