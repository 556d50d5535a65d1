set -o pipefail
export TMPDIR=/tmp
HEAD=0 WLS="grad grad_box grad_lunar" PHASES=0 TAG=r5b tools/gpu_round.sh || exit $?
O=gpurun_out/r5b
timeout -k 10 200 python tools/phase_prof.py --mode grad --scenario robocup --launches 3 > $O/phase_grad_robocup.json && timeout -k 10 200 python tools/phase_prof.py --mode grad --scenario box --launches 3 > $O/phase_grad_box.json && timeout -k 10 300 python tools/phase_prof.py --mode grad --scenario lunar --launches 3 > $O/phase_grad_lunar.json && echo phase ok
