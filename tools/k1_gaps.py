"""K = 1 RL loop (perf tooling): split the wall time per `env.step(1)` call
into step-kernel time and the gap to the next step kernel, from the
rocprofv3 kernel trace written by tools/gpu_k1.sh.

  python tools/k1_gaps.py <trace dir> [out.json]

Only the step kernels of the timed calls are used: the trace's step-kernel
dispatches after the first `skip` (warm-up) ones.  gap = start of launch
i + 1 - end of launch i (host submission, dispatch and the command
processor's turnaround between two back-to-back kernels on one stream)."""
import csv
import glob
import json
import os
import sys

import numpy as np


def main():
    d = sys.argv[1]
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "step_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    skip = 50  # k1_loop.py's warm-up calls
    rows = rows[skip:]
    st = np.array([r[0] for r in rows], dtype=np.float64)
    en = np.array([r[1] for r in rows], dtype=np.float64)
    dur = (en - st) / 1e3
    gap = (st[1:] - en[:-1]) / 1e3
    period = np.diff(st) / 1e3
    out = {
        "trace": os.path.relpath(path),
        "kernel": rows[0][2],
        "launches": len(rows),
        "kernel_us": {"mean": float(dur.mean()), "median": float(np.median(dur)), "p10": float(np.percentile(dur, 10)),
                      "p90": float(np.percentile(dur, 90))},
        "gap_us": {"mean": float(gap.mean()), "median": float(np.median(gap)), "p10": float(np.percentile(gap, 10)),
                   "p90": float(np.percentile(gap, 90))},
        "period_us": {"mean": float(period.mean()), "median": float(np.median(period))},
        "kernel_share_of_period": float(dur[:-1].sum() / (st[-1] - st[0]) * 1e3),
        "env_steps_per_s_from_trace": float(4096 / (period.mean() * 1e-6)),
    }
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
