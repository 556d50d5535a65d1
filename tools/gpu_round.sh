#!/bin/bash
# full GPU round: parity tests -> smoke -> benches -> rocprofv3 trace + PMC per
# scenario.  Every GPU step time-boxed; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/smoke.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --scenario lunar --cpu-seconds 8 > gpurun_out/bench_lunar.log 2>&1
rc=$?; echo "bench lunar rc=$rc"; tail -1 gpurun_out/bench_lunar.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode grad --steps 10 --warmup 2 --cpu-seconds 8 > gpurun_out/bench_grad.log 2>&1
rc=$?; echo "bench grad rc=$rc"; tail -1 gpurun_out/bench_grad.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
for sc in robocup lunar; do
  P=gpurun_out/prof_$sc; mkdir -p $P
  B="python bench.py --scenario $sc --steps 10 --warmup 2 --cpu-baseline off"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $B > $P/trace_bench.json 2> $P/trace.err || { tail $P/trace.err; exit 2; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/pmc_fetch -o run --output-format csv -- $B > /dev/null 2> $P/pmc1.err || { tail $P/pmc1.err; exit 3; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/pmc_write -o run --output-format csv -- $B > /dev/null 2> $P/pmc2.err || { tail $P/pmc2.err; exit 4; }
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $P/pmc_sq -o run --output-format csv -- $B > /dev/null 2> $P/pmc3.err || { tail $P/pmc3.err; exit 5; }
  echo "profile $sc ok"
done
timeout -k 10 200 python tools/phase_prof.py > gpurun_out/phase_robocup.json && timeout -k 10 200 python tools/phase_prof.py --scenario lunar > gpurun_out/phase_lunar.json && echo "phase ok"
