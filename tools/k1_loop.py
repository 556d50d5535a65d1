"""K = 1 RL loop (perf tooling): BatchedEnv(RoboCup 4096, autoreset).step(1)
called from Python, as an RL loop with per-step control would; prints the
wall rate and the per-launch HIP-event time (run under rocprofv3 by
tools/gpu_k1.sh to split kernel time and launch gaps)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import parallax_amd as pa  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    scen = pa.RoboCupEnv(batch=4096, perturb=True, device=dev)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    act = torch.zeros(4096, 2, device=dev)
    for _ in range(50):
        env.step(1)
    torch.cuda.synchronize()
    out = {}
    for name, fn in (("step", lambda: env.step(1)), ("step_action", lambda: env.step(1, action=act))):
        n = 2000
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        out[name] = {"env_steps_per_s": 4096 * n / wall, "us_per_call": wall / n * 1e6}
    # the kernel alone: HIP events around each launch (a separate pass)
    n = 500
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in evs:
        e0.record()
        env.step(1)
        e1.record()
    torch.cuda.synchronize()
    out["kernel_us_events"] = sum(a.elapsed_time(b) for a, b in evs) / n * 1e3
    # the host side alone: the same Python path with the library call stubbed
    real = pa._ffi.lib.cotix_eval
    pa._ffi.lib.cotix_eval = lambda *a: 0
    try:
        t0 = time.perf_counter()
        for _ in range(n):
            env.step(1)
        out["python_us_per_call_no_launch"] = (time.perf_counter() - t0) / n * 1e6
    finally:
        pa._ffi.lib.cotix_eval = real
    print(json.dumps(out))


if __name__ == "__main__":
    main()
