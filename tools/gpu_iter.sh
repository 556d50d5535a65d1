#!/bin/bash
# one perf iteration on the GPU box: (TESTS=1) every -m gpu test + smoke, the
# headline bench in both PRNG layouts (BENCH_LAYOUTS), an A/B of library builds
# (LIBS, REP alternations, SCS scenes, AB_LAYOUTS), then the per-phase cycle profile of the
# profiling build.  Each GPU step time-boxed; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-iter}
O=gpurun_out/$TAG; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/smoke.log; exit $rc; }
fi
for L in ${BENCH_LAYOUTS-legacy partitionable}; do
  timeout -k 10 300 python bench.py --extras off --cpu-baseline off --prng-layout $L > $O/bench_$L.json 2> $O/bench_$L.err
  rc=$?; [ $rc -eq 0 ] || { tail $O/bench_$L.err; exit $rc; }
  python -c "import json;d=json.load(open('$O/bench_$L.json'));print('bench $L', round(d['value']/1e6,1), 'M/s', round(d['roofline']['launch_ms'],4), 'ms')"
done
for r in $(seq 1 ${REP:-3}); do for L in $LIBS; do for SC in ${SCS:-robocup box}; do for PL in ${AB_LAYOUTS:-legacy}; do
  F=$O/ab_${L}_${SC}_${PL}_$r.json
  timeout -k 10 200 python bench.py --lib parallax_amd/_lib/$L --scenario $SC --prng-layout $PL --cpu-baseline off --extras off > $F 2> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$F'));print('ab $L $SC $PL', round(d['value']/1e6,1), round(d['roofline']['launch_ms'],4), d['config'].get('kernel_variant'))"
done; done; done; done
for SC in ${PHASE_SCS-robocup}; do
  timeout -k 10 200 python tools/phase_prof.py --scenario $SC > $O/phase_$SC.json 2> $O/phase.err || { tail $O/phase.err; exit 1; }
  python -c "import json;d=json.load(open('$O/phase_$SC.json'));print('phase $SC', round(d['cycles_per_wave_step_total']), {k:round(v['cycles_per_wave_step']) for k,v in d['phases'].items() if v['cycles_per_wave_step']>50})"
done
