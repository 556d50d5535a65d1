#!/bin/bash
# LunarLander per-phase cycles: airborne (bench start), without the
# broadphase, and dropped onto the terrain (in contact)
set -o pipefail
mkdir -p gpurun_out/llv
timeout -k 10 200 python tools/phase_prof.py --scenario lunar > gpurun_out/llv/air.json &&
timeout -k 10 200 python tools/phase_prof.py --scenario lunar --no-broadphase > gpurun_out/llv/air_nobp.json &&
timeout -k 10 200 python tools/phase_prof.py --scenario lunar --drop 6.3 > gpurun_out/llv/drop.json &&
timeout -k 10 200 python tools/phase_prof.py --scenario lunar --drop 6.3 --no-broadphase > gpurun_out/llv/drop_nobp.json
