"""K = 1 floor (perf tooling, run under rocprofv3 --kernel-trace): the
RoboCup 4096-env step kernel at one driver step per launch, in segments of
`N` back-to-back launches each: the RL-loop step (BatchedEnv.step(1)), the
same launch with every stage off (prologue + store only) and with Euler only,
and a trivial torch kernel.  `--parse <trace dir>` splits the trace into the
segments (in launch order) and prints the median kernel duration of each."""
import csv
import glob
import json
import os
import sys

import numpy as np

N, WARM = 300, 20
SEGS = ("env_step", "stages0", "euler")


def run():
    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import parallax_amd as pa

    dev = torch.device("cuda:0")
    scen = pa.RoboCupEnv(batch=4096, perturb=True, device=dev)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    w = scen.world
    fns = {
        "env_step": lambda: env.step(1),
        "stages0": lambda: w.step(1, 1e-2, 0, dyn_reset=scen.dyn_reset, resets=env.resets),
        "euler": lambda: w.step(1, 1e-2, 1, dyn_reset=scen.dyn_reset, resets=env.resets),
    }
    x = torch.zeros(4096, device=dev)
    for s in SEGS:
        for _ in range(WARM + N):
            fns[s]()
        torch.cuda.synchronize()
    for _ in range(N):
        x.add_(1.0)
    torch.cuda.synchronize()
    print("done")


def parse(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    step, other = [], []
    with open(path) as f:
        for r in csv.DictReader(f):
            t = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            (step if "step_kernel" in r["Kernel_Name"] else other).append((t, r["Kernel_Name"]))
    step.sort()
    out = {}
    for i, s in enumerate(SEGS):
        seg = step[i * (WARM + N) + WARM:(i + 1) * (WARM + N)]
        dur = np.array([(b - a) / 1e3 for (a, b), _ in seg])
        out[s + "_kernel_us"] = {"median": float(np.median(dur)), "mean": float(dur.mean()),
                                 "p10": float(np.percentile(dur, 10))}
    adds = [(b - a) / 1e3 for (a, b), n in other if "CUDAFunctor_add" in n or "add" in n.lower()]
    if adds:
        out["torch_add_kernel_us"] = float(np.median(adds[-N:]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
