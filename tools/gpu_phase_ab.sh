#!/bin/bash
# per-phase A/B of profiling-library variants (perf tooling): LIBS="a b" =
# parallax_amd/_lib/libcotix_amd_prof_<a>.so ..., ARGS = tools/phase_prof.py arguments
set -o pipefail
O=gpurun_out/${TAG:-phab}; mkdir -p $O
for r in 1 2; do for L in $LIBS; do
  timeout -k 10 200 python tools/phase_prof.py --lib parallax_amd/_lib/libcotix_amd_prof_$L.so $ARGS > $O/${L}_$r.json 2> $O/${L}_$r.err || { tail -3 $O/${L}_$r.err; exit 3; }
  python -c "
import json; d=json.load(open('$O/${L}_$r.json'))
for k in ('forward','backward'):
    if k in d:
        p=d[k]; print('$L', $r, k, round(p['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in p['phases'].items() if b['cycles_per_wave_step']>40})
if 'phases' in d: print('$L', $r, round(d['cycles_per_wave_step_total']), {a:round(b['cycles_per_wave_step']) for a,b in d['phases'].items() if b['cycles_per_wave_step']>40})"
done; done
