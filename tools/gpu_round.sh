#!/bin/bash
# full GPU round: parity tests -> smoke -> benches -> rocprofv3 trace + PMC per
# scenario -> per-phase cycles.  Every GPU step time-boxed; the chain stops at
# the first failure.  TAG names the output directory (gpurun_out/$TAG).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-round}
O=gpurun_out/$TAG; mkdir -p $O
if [ "${HEAD:-1}" = 1 ]; then  # HEAD=0: the profiles only (a second call)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/smoke.log; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench.json; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
fi
# workload key : bench arguments (lunar_contact: the landers on the terrain,
# driver steps 2560-3200, the stretch of the bench line's lunar_contact figure)
ALL=("robocup:--scenario robocup --warmup 2" "robocup_part:--scenario robocup --prng-layout partitionable --warmup 2" \
     "lunar:--scenario lunar --warmup 2" \
     "lunar_contact:--scenario lunar --warmup 40" "box:--scenario box --warmup 2" \
     "grad:--mode grad --scenario robocup --warmup 1" "grad_box:--mode grad --scenario box --warmup 1" \
     "grad_lunar:--mode grad --scenario lunar --warmup 1")
for wl in "${ALL[@]}"; do
  sc=${wl%%:*}
  [ -n "$WLS" ] && [[ " $WLS " != *" $sc "* ]] && continue  # WLS: a subset of the workloads
  sc=${wl%%:*}; args=${wl#*:}
  P=$O/prof_$sc; mkdir -p $P
  B="python bench.py $args --steps 10 --cpu-baseline off --extras off"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- $B > $P/trace_bench.json 2> $P/trace.err || { tail $P/trace.err; exit 2; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/pmc_fetch -o run --output-format csv -- $B > /dev/null 2> $P/pmc1.err || { tail $P/pmc1.err; exit 3; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/pmc_write -o run --output-format csv -- $B > /dev/null 2> $P/pmc2.err || { tail $P/pmc2.err; exit 4; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $P/pmc_sq -o run --output-format csv -- $B > /dev/null 2> $P/pmc3.err || { tail $P/pmc3.err; exit 5; }
  # the stall attribution: wave cycles = issuing (ACTIVE_INST_ANY) + parked on
  # waitcnt / barrier (WAIT_ANY) + issue-stalled (WAIT_INST_ANY, of it LDS)
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $P/pmc_stall -o run --output-format csv -- $B > /dev/null 2> $P/pmc4.err || { tail $P/pmc4.err; exit 6; }
  echo "profile $sc ok"
done
if [ "${PHASES:-1}" = 1 ]; then  # per-phase cycles (the tooling library of the same sources: COTIX_PHASE_PROF)
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
timeout -k 10 200 python tools/phase_prof.py --lib $L > $O/phase_robocup.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --scenario box > $O/phase_box.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --substeps 1 --launches 200 > $O/phase_k1.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --scenario lunar > $O/phase_lunar.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --scenario lunar --warmup 40 --launches 5 > $O/phase_lunar_settled.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario robocup --launches 3 > $O/phase_grad_robocup.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario box --launches 3 > $O/phase_grad_box.json && timeout -k 10 200 python tools/phase_prof.py --lib $L --mode grad --scenario lunar --launches 3 > $O/phase_grad_lunar.json && echo "phase ok"
fi
