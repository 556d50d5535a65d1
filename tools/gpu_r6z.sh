#!/bin/bash
# round-6 final build, part 1: the full GPU suite, smoke, the driver-style
# bench line, then kernel traces + PMC passes of the headline and config-5
# workloads (tools/gpu_round.sh); part 2 (PART=2): the other workloads'
# profiles and the per-phase cycles.  Every GPU step time-boxed inside
# gpu_round.sh; the chain stops at the first failure.
set -o pipefail
export TAG=${TAG:-r06z}
if [ "${PART:-1}" = 1 ]; then
  HEAD=1 PHASES=0 WLS="robocup grad grad_box lunar_contact" bash tools/gpu_round.sh
else
  HEAD=0 PHASES=1 WLS="robocup_part lunar box grad_lunar" bash tools/gpu_round.sh
fi
