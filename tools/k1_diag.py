"""K = 1 diagnosis (perf tooling): per-launch kernel time T(n) of the RoboCup
4096-env step at n = 1, 2, 4, 16, 64 driver steps per launch (HIP events),
fitted as fixed cost + n * per-step cost, for the plain autoreset step and the
RL-loop path (BatchedEnv.step with the observation written by the kernel)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import parallax_amd as pa  # noqa: E402


def timed(fn, n=200, warm=20):
    for _ in range(warm):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    t = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n))
    return 1e3 * t[len(t) // 2]


def main():
    dev = torch.device("cuda:0")
    scen = pa.RoboCupEnv(batch=4096, perturb=True, device=dev)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    w = scen.world
    out = {}
    for n in (1, 2, 4, 16, 64):
        out["env_step_n%d_us" % n] = timed(lambda: env.step(n))
        out["autoreset_n%d_us" % n] = timed(
            lambda: w.step(n, 1e-2, scen.stages, dyn_reset=scen.dyn_reset, resets=env.resets))
        out["plain_n%d_us" % n] = timed(lambda: w.step(n, 1e-2, scen.stages))
    # floors: a trivial torch kernel, the kernel with no stage / Euler only / keys only
    x = torch.zeros(4096, device=dev)
    out["torch_add_us"] = timed(lambda: x.add_(1.0))
    for name, st in (("stages0", 0), ("euler", 1), ("keys", 16), ("euler_keys", 17)):
        for n in (1, 64):
            out["%s_n%d_us" % (name, n)] = timed(lambda: w.step(n, 1e-2, st, dyn_reset=scen.dyn_reset,
                                                                  resets=env.resets))
    for k in ("env_step", "autoreset", "plain"):
        t1, t64 = out["%s_n1_us" % k], out["%s_n64_us" % k]
        s = (t64 - t1) / 63
        out["%s_fit" % k] = {"per_step_us": s, "fixed_us": t1 - s}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
