#!/bin/bash
# K = 1 RL-loop path (BatchedEnv.step(1) per call): rocprofv3 kernel trace of
# the k1 bench leg, to split kernel time from launch gaps.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-k1}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k1trace -o run --output-format csv -- python tools/k1_loop.py > $O/k1_loop.json 2> $O/k1.err || { tail $O/k1.err; exit 1; }
cat $O/k1_loop.json
