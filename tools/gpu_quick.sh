#!/bin/bash
# quick perf iteration: headline-style bench of one scenario + per-phase
# cycles (profiling build).  SC=robocup|lunar, TAG names gpurun_out/$TAG.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-quick}; SC=${SC:-lunar}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 200 python bench.py --scenario $SC --cpu-baseline off --extras off > $O/bench_$SC.json 2> $O/bench_$SC.err || { tail $O/bench_$SC.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_$SC.json'));print('$SC', round(d['value']/1e6,1), 'M env-steps/s', round(d['roofline']['launch_ms'],4), 'ms/launch')"
timeout -k 10 200 python tools/phase_prof.py --scenario $SC > $O/phase_$SC.json || exit 2
python - <<PY
import json
d=json.load(open('$O/phase_$SC.json'))
print(round(d['cycles_per_wave_step_total']), {k:round(v['cycles_per_wave_step']) for k,v in d['phases'].items() if v['cycles_per_wave_step']>50})
PY
