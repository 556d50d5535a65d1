#!/bin/bash
# round-5 check: the -m gpu suite, smoke, the full bench line, the K = 1 floor
# trace and the per-phase profiles (K = 64 and K = 1).  Time-boxed steps,
# stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5c}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/smoke.log; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
python tools/show_bench.py $O/bench.json 2>/dev/null || cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k1floor -o run --output-format csv -- python tools/k1_floor.py > $O/k1floor.out 2> $O/k1floor.err || { tail $O/k1floor.err; exit 1; }
python tools/k1_floor.py --parse $O/k1floor > $O/k1floor.json && cat $O/k1floor.json
timeout -k 10 200 python tools/phase_prof.py > $O/phase_robocup.json && timeout -k 10 200 python tools/phase_prof.py --substeps 1 --launches 200 > $O/phase_k1.json || exit 1
python -c "
import json
for f in ('phase_robocup','phase_k1'):
    d=json.load(open('$O/'+f+'.json')); print(f, round(d['cycles_per_wave_step_total']), {k:round(v['cycles_per_wave_step']) for k,v in d['phases'].items() if v['cycles_per_wave_step']>50})"
