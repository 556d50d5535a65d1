"""Config 1 (one LunarLander env, 10,000 driver steps in one launch) under
the envs-per-wave tiling given as argv[1] (default 4; perf tooling)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import parallax_amd as pa  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    ew = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ll = pa.LunarLander(batch=1, device=dev)
    ll.world.set_variant(ew)
    dyn0, keys0 = ll.world.dyn.clone(), ll.world.keys.clone()
    ts = []
    for _ in range(3):
        ll.world.dyn.copy_(dyn0)
        ll.world.keys.copy_(keys0)
        ll.world.err.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ll.world.step(10000, 1e-2, ll.stages)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(json.dumps({"ew": ew, "ms_per_10000": min(ts),
                      "env_steps_per_s": 10000 / (min(ts) * 1e-3),
                      "state_sum": float(torch.nan_to_num(ll.world.dyn).sum().item())}))


if __name__ == "__main__":
    main()
