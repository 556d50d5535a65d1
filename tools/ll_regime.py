"""LunarLander regime over the trajectory (perf tooling): per 64-step launch
of the bench workload (4096 envs), the fraction of envs in which some body
chose a contact partner (collider trace), and the mean lander height."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import parallax_amd as pa  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = 4096
    tk = pa.random.split(pa.random.PRNGKey(0, dev), B).contiguous()
    ck = pa.random.split(pa.random.PRNGKey(1, dev), B).contiguous()
    scen = pa.LunarLander(key=tk, batch=B, device=dev, collider_keys=ck)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    rows = []
    for launch in range(48):
        tr = {}
        env.step(64, trace=tr)
        ch = tr["chosen"]
        own = torch.arange(ch.shape[1], device=dev, dtype=ch.dtype)[None, :, None]
        frac = float((ch != own).any(1).any(0).float().mean().item())
        rows.append({"steps": 64 * (launch + 1), "contact_env_fraction": frac,
                     "lander_y_mean": float(scen.world.dyn[0, 1].mean().item()),
                     "lander_vy_mean": float(scen.world.dyn[0, 3].mean().item())})
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
