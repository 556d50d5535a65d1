#!/bin/bash
# instruction-issue / instruction-cache counters of the step kernel (perf
# tooling).  One rocprofv3 --pmc pass per counter group, each time-boxed;
# stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icache}; mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_ACTIVE_INST[A-Z_]*" $O/list_avail.txt | sort -u > $O/names.txt
echo "names: $(tr '\n' ' ' < $O/names.txt)"
for SC in robocup lunar; do
  B="python bench.py --scenario $SC --steps 10 --warmup 2 --cpu-baseline off"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d $O/${SC}_sq -o run --output-format csv -- $B > /dev/null 2> $O/${SC}_sq.err || { tail -3 $O/${SC}_sq.err; exit 3; }
  if grep -q "SQC_ICACHE_MISSES" $O/names.txt && grep -q "SQC_ICACHE_HITS" $O/names.txt; then
    timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $O/${SC}_sqc -o run --output-format csv -- $B > /dev/null 2> $O/${SC}_sqc.err || { tail -3 $O/${SC}_sqc.err; exit 4; }
  fi
  echo "$SC done"
done
