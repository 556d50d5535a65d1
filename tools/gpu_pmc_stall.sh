#!/bin/bash
# stall attribution of the step kernel: the SQ issue /
# wait buckets of the bench workload, one rocprofv3 --pmc pass per counter
# group (each within gfx950's 8 SQ slots), plus the counter list of the box.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-stall}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
SC=${SCS:-robocup}
for sc in $SC; do
  B="python bench.py --scenario $sc --warmup 2 --steps 10 --cpu-baseline off --extras off"
  P=$O/$sc; mkdir -p $P
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $P/pmc_stall -o run --output-format csv -- $B > /dev/null 2> $P/stall.err || { tail $P/stall.err; exit 3; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAVES -d $P/pmc_mix -o run --output-format csv -- $B > /dev/null 2> $P/mix.err || { tail $P/mix.err; exit 4; }
  echo "pmc $sc ok"
done
