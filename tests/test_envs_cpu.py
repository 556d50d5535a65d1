"""AbstractEnvironment.eval (cotix/_envs.py:37-132) on CPU: the product's
batched loop (parallax_amd.envs) over a world backed by the host emulation of
the step kernel, against the oracle's single-env restatement
(oracle/cotix_oracle/envs.py) -- rewards and end states bit for bit,
including envs frozen by is_done mid-NFE."""
import os
import subprocess
import sys

import numpy as np
import torch

import grad_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))


class EmuWorld:
    """AbstractWorld.forward through the kernel's host emulation (CPU tensors)."""

    def __init__(self, emu, lib, bodies, stages):
        self.emu, self.lib, self.stages = emu, lib, stages
        self.h, self.geom = emu.oracle_scene(lib, bodies)

    def forward(self, state, sig, dt):
        from parallax_amd import envs as E
        out = state.clone()
        dyn = out.dyn.numpy()
        keys = out.keys.numpy().view(np.uint32)
        err = out.err.numpy().view(np.uint32)
        act = np.ascontiguousarray(sig.apply(state, dt).numpy()[None], np.float32)
        P = self.emu.P_
        self.lib.emu_step(self.h, dyn.ctypes.data_as(P), keys.ctypes.data_as(P), err.ctypes.data_as(P),
                          self.geom.ctypes.data_as(P), 0, dyn.shape[2], 1, dt, self.stages,
                          act.ctypes.data_as(P), sig.body, None, None, 4)
        return E.WorldState(torch.from_numpy(dyn), torch.from_numpy(keys.view(np.int32)),
                            torch.from_numpy(err.view(np.int32)))


def _run(case, B, period, nfe, wfe):
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    import eval_cases as EC
    from parallax_amd import envs as E
    from cotix_oracle import envs as OE
    lib = emu.load()
    ab = case["ab"]
    world = EmuWorld(emu, lib, case["make"](), 1 | 4 | 16)
    S0 = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    state = E.WorldState(torch.from_numpy(S0.copy()),
                         torch.from_numpy(np.array(case["keys"], np.uint32).view(np.int32).copy()),
                         torch.zeros(B, dtype=torch.int32))
    env = E.AbstractEnvironment(world, state, EC.PDControl(ab), EC.XJudge(ab))
    out, reward = env.eval(period, nfe, wfe)
    done = 0
    for e in range(B):
        bodies = case["make"]()
        for b, row in zip(bodies, case["S0"][e]):
            b.set_dyn(row)
        (ob, okey), orew = OE.eval_env(case["step"], (bodies, np.asarray(case["keys"][e], np.uint32)),
                                       EC.OraclePD(ab), EC.OracleX(ab), period, nfe, wfe, GC.D0, ab)
        want = np.array([b.dyn() for b in ob], np.float32)
        got = out.state.dyn[:, :, e].numpy()
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (e, got, want)
        assert np.array_equal(out.state.keys[e].numpy().view(np.uint32), okey)
        r = reward[e].numpy()
        assert (np.isnan(r) and np.isnan(orew)) or r.view(np.uint32) == np.float32(orew).view(np.uint32), (e, r, orew)
        done += int(want[ab, 0] > 1.2)
    return done


def test_eval_box_world_matches_oracle():
    B = 8
    case = GC.box_case(B, 1, seed=5)
    case["S0"][1, case["ab"], 0] = 1.5  # done before the first NFE: frozen at its start state
    done = _run(case, B, 0.6, 3, 10)
    assert done >= 3  # several envs finish mid-NFE (seed 5), one from the start


def test_eval_robocup_matches_oracle():
    B = 6
    case = GC.robocup_case(B, 1)
    _run(case, B, 0.2, 2, 5)
