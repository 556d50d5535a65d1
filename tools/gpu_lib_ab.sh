#!/bin/bash
# A/B of library builds (perf tooling): LIBS="a.so b.so" under parallax_amd/_lib,
# alternated REPS times: the K = 1 RL loop (tools/k1_loop.py) and the per-launch fit
# (tools/k1_diag.py).  Time-boxed steps, stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-libab}; mkdir -p $O
for r in $(seq ${REPS:-3}); do
  for L in $LIBS; do
    COTIX_AMD_LIB=$PWD/parallax_amd/_lib/$L timeout -k 10 120 python tools/k1_loop.py > $O/${L}_k1_$r.json 2> $O/${L}_k1_$r.err || { tail -5 $O/${L}_k1_$r.err; exit 3; }
    COTIX_AMD_LIB=$PWD/parallax_amd/_lib/$L timeout -k 10 120 python tools/k1_diag.py > $O/${L}_diag_$r.json 2> $O/${L}_diag_$r.err || { tail -5 $O/${L}_diag_$r.err; exit 4; }
    python -c "
import json,sys
k=json.load(open('$O/${L}_k1_$r.json')); d=json.load(open('$O/${L}_diag_$r.json'))
print('$L', $r, 'k1 %.1f M %.2f us/call kernel %.2f us' % (k['step']['env_steps_per_s']/1e6, k['step']['us_per_call'], k['kernel_us_events']),
      'n64 %.1f us (%.1f M)' % (d['autoreset_n64_us'], 4096*64/d['autoreset_n64_us']), 'stages0_n1 %.2f torch %.2f' % (d['stages0_n1_us'], d['torch_add_us']))"
  done
done
