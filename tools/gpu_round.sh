#!/bin/bash
# full GPU round: parity tests -> smoke -> bench -> rocprofv3 trace + PMC.
# Every step time-boxed; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/smoke.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scenario lunar --cpu-seconds 8 > gpurun_out/bench_lunar.log 2>&1
rc=$?; echo "bench lunar rc=$rc"; tail -1 gpurun_out/bench_lunar.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --cpu-baseline off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- $B > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace.err || { tail gpurun_out/prof/trace.err; exit 2; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc1.err || { tail gpurun_out/prof/pmc1.err; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc2.err || { tail gpurun_out/prof/pmc2.err; exit 4; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/prof/pmc_sq -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc3.err || { tail gpurun_out/prof/pmc3.err; exit 5; }
echo "profile ok"
