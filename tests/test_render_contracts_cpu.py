"""Render export and contract checks on CPU.

* The render kernel's device code (cotix_body.h, host build in tests/emu)
  + the host command list (parallax_amd.render) must issue the Painter
  calls of the reference's env.draw(painter) -- restated in
  oracle/cotix_oracle/render.py -- with bit-identical coordinates, for
  RoboCup (fill + outline passes, colours) and LunarLander (polygons
  re-sorted after the transform, default colours, the two red lines).
* parallax_amd.contracts: pre/post conditions and class invariants with the
  reference's API, per-env NaN guarding and error bits.
"""
import os
import subprocess
import sys
import types

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(HERE, "emu"))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    import emu
    lib = emu.load()
    lib.emu_render.argtypes = [emu.P_] * 3 + [emu.ctypes.c_int, emu.ctypes.c_int, emu.P_]
    return emu, lib


def _pa_struct(obodies):
    """Host-side body list with the oracle bodies' part structure (the
    command list only needs part kinds and vertex counts)."""
    import parallax_amd.shapes as S
    from cotix_oracle import geometry as G
    out = []
    for b in obodies:
        parts = []
        for p in b.parts:
            if isinstance(p, G.Circle):
                parts.append(S.Circle(1.0, (0.0, 0.0)))
            elif isinstance(p, G.AABB):
                parts.append(S.AABB((0.0, 0.0), (1.0, 1.0)))
            else:
                parts.append(S.Polygon(torch.zeros(len(p.vertices_), 2)))
        out.append(types.SimpleNamespace(shape=types.SimpleNamespace(parts=parts)))
    return out


def _norm(calls):
    f = np.float32
    out = []
    for c in calls:
        if c[0] == "circle":
            out.append(("circle", (f(c[1][0]), f(c[1][1])), f(c[2]), tuple(c[3])))
        elif c[0] == "line":
            out.append(("line", (f(c[1][0]), f(c[1][1])), (f(c[2][0]), f(c[2][1])), tuple(c[3])))
        else:
            out.append(c)
    return [tuple(np.array(x, dtype=object).tolist() if isinstance(x, np.ndarray) else x for x in c) for c in out]


def _same_calls(got, want):
    assert len(got) == len(want)
    for g, w in zip(_norm(got), _norm(want)):
        assert g[0] == w[0]
        if g[0] == "next":
            continue
        ga = np.array([v for t in g[1:-1] for v in (t if isinstance(t, tuple) else (t,))], np.float32)
        wa = np.array([v for t in w[1:-1] for v in (t if isinstance(t, tuple) else (t,))], np.float32)
        assert np.array_equal(ga.view(np.uint32), wa.view(np.uint32)), (g, w)
        assert g[-1] == w[-1], (g, w)


def _emu_prims(emu, lib, obodies, dyn, geom, gstride):
    h, _ = emu.oracle_scene(lib, obodies)
    B = dyn.shape[2]
    n = lib.emu_render(h, dyn.ctypes.data_as(emu.P_), geom.ctypes.data_as(emu.P_), gstride, B, None)
    prims = np.zeros((B, max(n, 1), 4), np.float32)
    assert lib.emu_render(h, dyn.ctypes.data_as(emu.P_), geom.ctypes.data_as(emu.P_), gstride, B,
                          prims.ctypes.data_as(emu.P_)) == n
    return prims


def test_render_robocup_vs_reference_draw(emu_lib):
    emu, lib = emu_lib
    import parallax_amd.render as R
    from parallax_amd.scenarios import RoboCupEnv
    from cotix_oracle import physics as P
    from cotix_oracle import render as OR
    tr = np.load(os.path.join(GOLD, "robocup_trace.npz"))
    ob = P.robocup_bodies()
    _, geom = emu.oracle_scene(lib, ob)
    cmds = R.commands_bodies(_pa_struct(ob), RoboCupEnv.colors, RoboCupEnv.edge_colors)
    for t in (0, 5, 12):
        dyn = np.ascontiguousarray(tr["dyn"][t].transpose(1, 2, 0))
        prims = _emu_prims(emu, lib, ob, dyn, geom, 0)
        for e in range(dyn.shape[2]):
            bodies = P.robocup_bodies()
            for i, b in enumerate(bodies):
                b.set_dyn(tr["dyn"][t][e, i])
            p = R.RecordingPainter()
            R.replay(p, cmds, prims, e)
            _same_calls(p.calls, OR.robocup_draw(bodies))


def test_render_lunar_vs_reference_draw(emu_lib):
    emu, lib = emu_lib
    import parallax_amd.render as R
    from cotix_oracle import physics as P
    from cotix_oracle import render as OR
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    obs = [P.lunar_lander_bodies(k) for k in tr["terrain_keys"]]
    geom = np.ascontiguousarray(np.stack([emu.oracle_scene(lib, ob)[1] for ob in obs]).astype(np.float32))
    red = (255, 0, 0)
    cmds = R.commands_bodies(_pa_struct(obs[0]), extra_lines=[((-2, -1.8), (-2, -1.0), red), ((2, -1.8), (2, -1.0), red)])
    for t in (0, 7, 12):
        dyn = np.ascontiguousarray(tr["dyn"][t].transpose(1, 2, 0))
        prims = _emu_prims(emu, lib, obs[0], dyn, geom, geom.shape[1])
        for e in range(dyn.shape[2]):
            bodies = P.lunar_lander_bodies(tr["terrain_keys"][e])
            for i, b in enumerate(bodies):
                b.set_dyn(tr["dyn"][t][e, i])
            p = R.RecordingPainter()
            R.replay(p, cmds, prims, e)
            _same_calls(p.calls, OR.lunar_lander_draw(bodies))


def test_check_state_device_code(emu_lib):
    emu, lib = emu_lib
    lib.emu_check_state.argtypes = [emu.P_, emu.ctypes.c_int, emu.ctypes.c_int, emu.P_]
    dyn = np.zeros((5, 6, 16), np.float32)
    dyn[2, 3, 4] = np.nan
    dyn[0, 0, 9] = np.inf
    dyn[4, 5, 15] = -np.inf
    err = np.zeros(16, np.uint32)
    err[1] = 1
    lib.emu_check_state(dyn.ctypes.data_as(emu.P_), 5, 16, err.ctypes.data_as(emu.P_))
    want = np.zeros(16, np.uint32)
    want[1] = 1
    want[[4, 9, 15]] |= 4
    assert np.array_equal(err, want)


# ---------------------------------------------------------------------------
# contracts (host logic)
# ---------------------------------------------------------------------------
def test_pre_and_post_condition_guard_failing_envs():
    from parallax_amd import contracts as C

    @C.pre_condition(lambda x, y: x > 0)
    def f(x, y):
        return x + y

    x = torch.tensor([1.0, -1.0, 2.0])
    got = f(x, torch.tensor([10.0, 10.0, 10.0]))
    assert torch.isnan(got[1]) and got[0] == 11.0 and got[2] == 12.0

    @C.post_condition(lambda r: r < 5)
    def g(x):
        return x * 2

    got = g(torch.tensor([1.0, 3.0]))
    assert got[0] == 2.0 and torch.isnan(got[1])

    @C.post_condition(lambda r, x: r > x, provide_input=True)
    def h(x):
        return x - 1

    assert torch.isnan(h(torch.tensor([0.0]))).all()


def test_error_if_worldstate_sets_error_bit():
    from parallax_amd import contracts as C
    from parallax_amd.envs import WorldState
    s = WorldState(torch.ones(5, 6, 4), torch.zeros(4, 2, dtype=torch.int32), torch.tensor([0, 1, 0, 0], dtype=torch.int32))
    out = C.error_if(s, torch.tensor([False, True, False, True]))
    assert torch.isnan(out.dyn[..., 1]).all() and torch.isnan(out.dyn[..., 3]).all()
    assert (out.dyn[..., 0] == 1).all() and (out.dyn[..., 2] == 1).all()
    assert out.err.tolist() == [0, 1 | C.ERR_CONTRACT, 0, C.ERR_CONTRACT]


def test_class_invariant_semantics():
    """As in the reference, __invariant__() returning True is the failure
    (it is eqx.error_if's condition); annotations are type-checked."""
    from parallax_amd import contracts as C

    @C.class_invariant
    class Box:
        size: float

        def __init__(self, v):
            self.size = 1.0
            self.v = v

        def __invariant__(self):
            return self.v < 0

        def total(self):
            return self.v.sum()

    b = Box(torch.tensor([1.0, -2.0, 3.0]))
    assert torch.isnan(b.total())
    assert torch.isnan(b.v[1]) and b.v[0] == 1.0
    ok = Box(torch.tensor([1.0, 2.0]))
    assert ok.total() == 3.0
    bad = Box(torch.tensor([1.0]))
    bad.size = "big"
    with pytest.raises(TypeError):
        bad.total()
