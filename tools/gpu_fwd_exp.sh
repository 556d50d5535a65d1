#!/bin/bash
# config-5 forward save-phase experiments (perf tooling): phase cycles of the
# rollout forward with the tooling library, the save's tape stores (128) and
# state / key stores (256) skipped -- timing only, no backward after a skip
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fwdexp}; mkdir -p $O
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
for sc in ${SCS:-robocup box}; do
for sk in ${SKIPS:-0 128 256 384}; do
  timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario $sc --launches 3 --fwd-skip $sk > $O/${sc}_$sk.json 2> $O/${sc}_$sk.err || { tail -5 $O/${sc}_$sk.err; exit 3; }
  python -c "
import json; d=json.load(open('$O/${sc}_$sk.json')); p=d['forward']
print('$sc', $sk, round(p['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in p['phases'].items() if b['cycles_per_wave_step']>40})"
done; done
