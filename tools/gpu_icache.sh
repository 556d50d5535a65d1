#!/bin/bash
# instruction / scalar cache PMC passes of the config-5 kernels and the plain
# step (perf tooling): SQC_ICACHE_* and SQC_DCACHE_* per kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icache}; mkdir -p $O
for wl in "grad:--mode grad --scenario robocup --warmup 1" "robocup:--scenario robocup --warmup 2" "grad_box:--mode grad --scenario box --warmup 1"; do
  sc=${wl%%:*}; args=${wl#*:}
  B="python bench.py $args --steps 3 --cpu-baseline off --extras off"
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/${sc}_ic -o run --output-format csv -- $B > /dev/null 2> $O/${sc}_ic.err || { tail $O/${sc}_ic.err; exit 3; }
  timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $O/${sc}_dc -o run --output-format csv -- $B > /dev/null 2> $O/${sc}_dc.err || { tail $O/${sc}_dc.err; exit 4; }
  echo "$sc ok"
done
