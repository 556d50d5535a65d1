"""Per-wave timeline of one K = 1 launch (perf tooling; the profiling build,
tools/phase_prof.py --build): RoboCup 4096 envs, BatchedEnv.step(1) in a
loop, then the last launch's per-wave s_memrealtime stamps (100 MHz,
chip-wide) -- kernel entry, state loaded, after the workgroup barrier, end
after the stores completed -- summarized against the earliest entry:
  python tools/k1_stamps.py [--lib path] [--steps K]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
LIB = os.path.join(ROOT, "parallax_amd", "_lib", "libcotix_amd_prof.so")


def pct(x):
    x = np.asarray(x, np.float64)
    return {"min": float(x.min()), "p50": float(np.median(x)), "p90": float(np.percentile(x, 90)),
            "max": float(x.max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--launches", type=int, default=300)
    a = ap.parse_args()
    os.environ["COTIX_AMD_LIB"] = os.path.abspath(a.lib)
    sys.path.insert(0, ROOT)
    import torch
    import parallax_amd as pa
    f = pa._ffi.lib.cotix_phase_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    B = 4096
    scen = pa.RoboCupEnv(batch=B, perturb=True, device=dev)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    for _ in range(50):
        env.step(a.steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.launches):
        env.step(a.steps)
    torch.cuda.synchronize()
    call_us = (time.perf_counter() - t0) / a.launches * 1e6
    waves = B // 4
    buf = (ctypes.c_ulonglong * (4 * waves))()
    n = f(buf, 4 * waves)
    assert n == 4 * waves, n
    s = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 4).astype(np.int64)
    t = (s - s[:, 0].min()) * 0.01  # microseconds from the first wave's entry
    out = {
        "steps_per_launch": a.steps, "loop_us_per_call": call_us,
        "span_us": float(t[:, 3].max()),
        "entry_us": pct(t[:, 0]),
        "prologue_us": pct(t[:, 1] - t[:, 0]),  # table copy + state load (+ the one-step key chain)
        "barrier_wait_us": pct(t[:, 2] - t[:, 1]),
        "body_us": pct(t[:, 3] - t[:, 2]),  # the phases and the completed stores
        "end_us": pct(t[:, 3]),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
