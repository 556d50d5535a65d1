"""Per-env body parameters on CPU (COTIX_SCENE_PER_ENV_BODY_PARAMS): the
kernel's host emulation == the C port fed the same per-env parameters, bit
for bit with the collider's choices, at every envs-per-wave tiling; the
pytree adapter lays a vmapped pytree whose parameter leaves vary out as that
scene (tests/penv_cases.py).  The GPU side: tests/test_gpu_pytree.py."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "emu"))

import penv_cases as PC  # noqa: E402
import ref_standins as RS  # noqa: E402

STAGES = 1 | 2 | 4 | 8 | 16 | 32


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.fixture(scope="module")
def libs():
    import emu
    from cotix_oracle import cport
    assert os.path.exists(cport.LIB)
    return emu, emu.load(), cport, cport.load()


@pytest.mark.parametrize("EW", [1, 4, 8])
def test_emu_per_env_params_vs_cport(libs, EW):
    emu, lib, cport, clib = libs
    B, T = 12, 40
    obs = PC.lunar_penv_bodies(B)
    h, g0 = emu.oracle_scene(lib, obs[0], per_env_params=True)
    sc = cport.Scene(clib, obs[0])
    G = sc.set_per_env_params(True)
    geom = PC.rows(lambda ob: cport.Scene(clib, ob).geom, obs)
    assert geom.shape == (B, G) and G == len(g0) + 16
    dyn, keys = PC.state(obs)
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    gch, gcl = emu.step_ex(lib, h, *got, geom, G, T, STAGES, 4, E=EW)
    wch, wcl = sc.step_ex(*want, T, STAGES & ~32, geom=geom, trace=True)
    assert (wch != np.arange(4)[None, :, None]).sum() > B  # resolutions happen (the ground picks a leg)
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])
    for a, b in zip(got[1:], want[1:]):
        assert np.array_equal(a, b)
    # the parameters matter: the shared-parameter scene (env 0's) differs
    ref = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    sc0 = cport.Scene(clib, obs[0])
    sc0.step(*ref, T, STAGES & ~32, geom=geom[:, :len(g0)])
    assert not same_f32(ref[0], want[0])


def test_pytree_per_env_params_layout(libs):
    """World.from_bodies of a vmapped pytree whose mass / inertia / elasticity
    / friction leaves vary: per-env scene, the C port's rows, generic kernel."""
    import parallax_amd as pa
    emu, lib, cport, clib = libs
    obs = PC.lunar_penv_bodies(5)
    w = pa.World.from_bodies(RS.stack([RS.from_oracle(ob) for ob in obs]), device="cpu")
    assert w.scene.per_env_params and w.B == 5
    assert w.scene.variant()["specialization"] == "generic"
    want = PC.rows(lambda ob: cport.Scene(clib, ob).geom, obs)
    assert w.geom.shape == want.shape and np.array_equal(w.geom.numpy().view(np.uint32), want.view(np.uint32))
    assert torch.equal(w.bodies[0].mass, torch.tensor([ob[0].mass for ob in obs]))
