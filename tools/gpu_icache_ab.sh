#!/bin/bash
# instruction-cache and issue-wait counters of the step kernel for two
# library builds (perf tooling): LIBS="a.so b.so", ARGS = bench arguments.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icab}; mkdir -p $O
for L in $LIBS; do
  B="python bench.py $ARGS --cpu-baseline off --extras off"
  COTIX_AMD_LIB=$PWD/parallax_amd/_lib/$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $O/${L}_sqc -o run --output-format csv -- $B > /dev/null 2> $O/${L}_sqc.err || { tail -3 $O/${L}_sqc.err; exit 3; }
  COTIX_AMD_LIB=$PWD/parallax_amd/_lib/$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU -d $O/${L}_sq -o run --output-format csv -- $B > /dev/null 2> $O/${L}_sq.err || { tail -3 $O/${L}_sq.err; exit 4; }
  python - $O $L <<'PY'
import csv, sys
from collections import defaultdict
O, L = sys.argv[1], sys.argv[2]
agg = defaultdict(list)
for d in ("sqc", "sq"):
    for r in csv.DictReader(open("%s/%s_%s/run_counter_collection.csv" % (O, L, d))):
        if "step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(L, {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
done
