#!/bin/bash
# differentiable rollout on the GPU: parity tests, bench (config 5), profile
set -o pipefail
mkdir -p gpurun_out/prof_grad
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode grad --steps 10 --warmup 2 > gpurun_out/bench_grad.log 2>&1
rc=$?; echo "bench grad rc=$rc"; tail -2 gpurun_out/bench_grad.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_grad/trace -o run --output-format csv -- python bench.py --mode grad --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/prof_grad/bench.json 2> gpurun_out/prof_grad/trace.err || { tail gpurun_out/prof_grad/trace.err; exit 2; }
echo "profile ok"
