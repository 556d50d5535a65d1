#!/bin/bash
# gradient parity subset + config-5 benches + forward/backward phase passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6b}; mkdir -p $O
TAG=$TAG bash tools/gpu_grad_quick.sh || exit $?
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
for sc in robocup box lunar; do
  timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario $sc --launches 3 > $O/phase_grad_$sc.json 2> $O/phase_grad_$sc.err || { tail -5 $O/phase_grad_$sc.err; exit 4; }
  python -c "
import json; d=json.load(open('$O/phase_grad_$sc.json'))
for k in ('forward','backward'):
    p=d[k]; print('$sc', k, round(p['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in p['phases'].items() if b['cycles_per_wave_step']>40})"
done
