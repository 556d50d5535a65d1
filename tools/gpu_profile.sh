#!/bin/bash
# tuning sweep + rocprofv3 kernel trace/stats + PMC passes (separate runs,
# --pmc never combined with other trace domains).  Stops at first failure.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-r01}
B="python bench.py --steps 10 --warmup 2 --cpu-baseline off"
for E in 8 16 32; do
  COTIX_ENVS_PER_BLOCK=$E timeout -k 10 120 $B > gpurun_out/prof/sweep_E$E.json 2>/dev/null || exit 1
  echo "E=$E $(python -c "import json;d=json.load(open('gpurun_out/prof/sweep_E$E.json'));print(d['value'], d['roofline']['launch_ms'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- $B > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace.err || { tail gpurun_out/prof/trace.err; exit 2; }
echo trace ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc1.err || { tail gpurun_out/prof/pmc1.err; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc2.err || { tail gpurun_out/prof/pmc2.err; exit 4; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/prof/pmc_sq -o run --output-format csv -- $B > /dev/null 2> gpurun_out/prof/pmc3.err || { tail gpurun_out/prof/pmc3.err; exit 5; }
echo pmc ok
find gpurun_out/prof -name "*.csv" | head -20
