#!/bin/bash
# round-6 final build: per-phase cycles (tooling library, one-wave kernels:
# tools/phase_prof.py sets COTIX_KEY_HELPER=0 / COTIX_SPLIT_BWD=0); each step
# time-boxed, chained with && (stops at the first failure)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
L=parallax_amd/_lib/libcotix_amd_prof_tool.so
timeout -k 10 150 python tools/phase_prof.py --lib $L > $O/phase_robocup.json 2> $O/phase_robocup.err && \
timeout -k 10 150 python tools/phase_prof.py --lib $L --scenario lunar --warmup 40 --launches 5 > $O/phase_lunar_settled.json 2> $O/phase_lunar_settled.err && \
timeout -k 10 150 python tools/phase_prof.py --lib $L --mode grad --scenario robocup --launches 3 > $O/phase_grad_robocup.json 2> $O/phase_grad_robocup.err && echo "phase ok"
