"""GPU parity at the bench's sizes in the regimes its secondary figures time
(through the C-ABI, every env vs the C port of the oracle, bit for bit --
state, keys, error bits, restarts and every contact choice):

* LunarLander 4096 envs SETTLED on the terrain: driver steps 2560-2624, the
  stretch the bench's lunar_contact figure times (after 40 launches of 64
  steps; tools/ll_regime.py: first touch-down ~770, settled from ~2500),
  where GJK / EPA / the edge contact points run for most envs;
* the box world (pa.BoxWorld, finite dynamics, the bench's finite_scene and
  grad_box workloads) at 4096 envs, 2 launches x 16 fused steps.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from test_gpu_parity import diff_report, same_f32  # noqa: E402


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a visible GPU (torch.cuda.is_available() is False)")
    return torch


@pytest.fixture(scope="module")
def cport_lib():
    from cotix_oracle import cport
    assert os.path.exists(cport.LIB), "oracle C port %s missing: build it before the GPU run" % cport.LIB
    return cport, cport.load()


def _compare(torch, w, resets, dyn, keys, err, want_resets, trc, wch, wcl):
    torch.cuda.synchronize()
    assert np.array_equal(trc["chosen"].cpu().numpy(), wch), "chosen"
    assert np.array_equal(trc["cells"].cpu().numpy(), wcl), "cells"
    got = w.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(w.err.cpu().numpy().view(np.uint32), err)
    if resets is not None:
        assert np.array_equal(resets.cpu().numpy().view(np.uint32), want_resets)


def test_lunar_4096_settled_regime_vs_cport(torch_cuda, cport_lib):
    """The bench's lunar_contact workload: make_scenario("lunar") at 4096
    envs, BatchedEnv with autoreset, 40 x 64 driver steps on the GPU, then
    ONE 64-step launch compared with the C port started from the same state
    (terrain per env, broadphase on, restarts from the reset state)."""
    torch = torch_cuda
    import bench
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    cport, lib = cport_lib
    B = 4096
    scen = bench.make_scenario(pa, "lunar", "cuda", B)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    for _ in range(40):
        env.step(64)
    w = env.world
    dyn = np.ascontiguousarray(w.dyn.cpu().numpy())
    keys = np.ascontiguousarray(w.keys.cpu().numpy().view(np.uint32))
    err = np.ascontiguousarray(w.err.cpu().numpy().view(np.uint32))
    geom = np.ascontiguousarray(w.geom.cpu().numpy())
    rst = np.ascontiguousarray(scen.dyn_reset.cpu().numpy())
    want_resets = np.ascontiguousarray(env.resets.cpu().numpy().view(np.uint32))
    trc = {}
    env.step(64, trace=trc)
    sc = cport.Scene(lib, P.lunar_lander_bodies(prng.split(prng.PRNGKey(0), B)[0]))
    wch, wcl = sc.step_ex(dyn, keys, err, 64, cport.STAGES_LUNAR, geom, None, 0, rst, want_resets, trace=True,
                          nthreads=16)
    _compare(torch, w, env.resets, dyn, keys, err, want_resets, trc, wch, wcl)
    # the regime: most envs' bodies choose a contact partner in this stretch
    own = np.arange(4)[None, :, None]
    assert (wch != own).any(1).any(0).mean() > 0.5
    assert (wcl >= 0).sum() > 64 * B  # polygon contacts with a contact point, every step


def _oracle_bodies(bodies):
    """The oracle's Body objects of host AnyBody objects (circle / AABB parts)."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    out = []
    for b in bodies:
        parts = []
        for p in b.shape.parts:
            g = p.local_geometry().numpy()
            if p.type_id == 0:
                parts.append(G.Circle(g[0], (g[1], g[2])))
            else:
                parts.append(G.AABB((g[0], g[1]), (g[2], g[3])))
        m, i, e, f = b.params()
        out.append(P.Body(parts, mass=m, inertia=i, elasticity=e, friction_coefficient=f))
    return out


def test_box_world_4096_vs_cport(torch_cuda, cport_lib):
    """pa.BoxWorld at 4096 envs (the finite_scene / grad_box workload): 2
    launches x 16 fused steps, every env vs the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    B = 4096
    bw = pa.BoxWorld(batch=B, device="cuda")
    w = bw.world
    dyn = np.ascontiguousarray(w.dyn.cpu().numpy())
    keys = np.ascontiguousarray(w.keys.cpu().numpy().view(np.uint32))
    err = np.zeros(B, np.uint32)
    sc = cport.Scene(lib, _oracle_bodies(bw.bodies))
    assert same_f32(sc.geom, w.geom.cpu().numpy())
    for q in range(2):
        trc = {}
        w.step(16, 1e-2, bw.stages, trace=trc)
        wch, wcl = sc.step_ex(dyn, keys, err, 16, cport.STAGES_ROBOCUP, trace=True, nthreads=16)
        _compare(torch, w, None, dyn, keys, err, None, trc, wch, wcl)
    assert np.isfinite(dyn).all()  # finite dynamics: every env, every word
    assert (wcl >= 0).sum() > B and (wch != np.arange(7)[None, :, None]).any()
