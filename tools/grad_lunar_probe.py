"""grad_lunar cost split (tooling): the settled-LunarLander rollout's forward
with and without the broadphase stage, and the backward (which re-plays
without it), kernel times by HIP events."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import parallax_amd as pa  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / n


def main():
    B, T = 4096, 64
    ll = pa.LunarLander(batch=B)
    st = pa._ffi.STAGES_LUNAR | pa._ffi.STAGE_BROADPHASE
    for _ in range(40):
        ll.world.step(64, 1e-2, st)
    w = ll.world
    d0, k0 = w.dyn.clone(), w.keys.clone()
    acts = torch.randn(T, B, 2, device="cuda") * 0.1
    wt = np.zeros(24, np.float32)
    wt[0] = 1.0
    out = {}
    saved = {}

    def fwd(stages):
        def f():
            w.dyn.copy_(d0)
            w.keys.copy_(k0)
            w.err.zero_()
            saved["s"] = pa.rollout_forward(w, acts, 0, wt, stages=stages)[1]
        return f
    out["fwd_bp_ms"] = timed(fwd(st))
    out["fwd_nobp_ms"] = timed(fwd(pa._ffi.STAGES_LUNAR))
    out["bwd_ms"] = timed(lambda: pa.rollout_backward(w, saved["s"]))
    out["step_mode0_bp_ms"] = timed(lambda: w.step(64, 1e-2, st))
    out["step_mode0_nobp_ms"] = timed(lambda: w.step(64, 1e-2, pa._ffi.STAGES_LUNAR))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
