#!/bin/bash
# one perf iteration on the GPU box: parity tests, bench + per-phase profile
# for envs-per-wave EWS (default "4 2"), each GPU step time-boxed; stops at
# the first failure.  TAG names the output files.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-iter}
EWS=${EWS:-"4 2"}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for E in $EWS; do for SC in robocup lunar; do
  COTIX_ENVS_PER_WAVE=$E timeout -k 10 120 python bench.py --scenario $SC --steps 20 --warmup 3 --cpu-baseline off > $O/bench_${SC}_EW$E.json 2> $O/bench_${SC}_EW$E.err || { tail $O/bench_${SC}_EW$E.err; exit 1; }
  echo "$SC EW=$E $(python -c "import json;d=json.load(open('$O/bench_${SC}_EW$E.json'));print('%.4g'%d['value'], 'launch_ms %.4g'%d['roofline']['launch_ms'])")"
  [ "$E" = 4 ] || continue  # the profiling build has the EW=4 tiling only
  COTIX_ENVS_PER_WAVE=$E timeout -k 10 120 python tools/phase_prof.py --scenario $SC > $O/phase_${SC}_EW$E.json 2> $O/phase.err || { tail $O/phase.err; exit 1; }
  python -c "import json;d=json.load(open('$O/phase_${SC}_EW$E.json'));print(' ', round(d['cycles_per_wave_step_total']), {k:round(v['cycles_per_wave_step']) for k,v in d['phases'].items()})"
done; done
