"""Kernel-logic parity on CPU: the fused step kernel's phase code
(parallax_amd/csrc/cotix_kernel.h), compiled for the host by the test-only
emulation harness (tests/emu), must reproduce the golden oracle traces bit
for bit -- the same bar as the GPU tests -- for every envs-per-wave tiling,
including the collider's contact choices (j* per body and the winning
candidate of every all_contacts cell, cotix/_colliders.py:208-295)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(HERE, "emu"))
sys.path.insert(0, GOLD)


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    import emu
    return emu, emu.load()


def _build_cport():
    """The oracle's C port (make -C oracle): built here when missing -- a
    missing checker is never a skip."""
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "..", "oracle")], check=True)


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def run_trace(emu, lib, bodies, geom_rows, tr, stages, EW, per_env_geom):
    h, geom = emu.oracle_scene(lib, bodies)
    B = tr["dyn"].shape[1]
    T = tr["err"].shape[0]
    if per_env_geom:
        geom = np.ascontiguousarray(np.stack(geom_rows).astype(np.float32))
        gstride = geom.shape[1]
    else:
        gstride = 0
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(np.uint32)
    err = np.zeros(B, np.uint32)
    nb = len(bodies)
    for t in range(T):
        ch, cl = emu.step_ex(lib, h, dyn, keys, err, geom, gstride, 1, stages, nb, E=EW)
        assert np.array_equal(ch[0].T, tr["chosen"][t]), "chosen step %d" % t
        assert np.array_equal(cl[0].transpose(2, 0, 1), tr["cells"][t]), "cells step %d" % t
        got = dyn.transpose(2, 0, 1)
        assert same_f32(got, tr["dyn"][t + 1]), "step %d" % t
        assert np.array_equal(keys, tr["keys"][t + 1]), "keys step %d" % t
        assert np.array_equal(err, np.bitwise_or.reduce(tr["err"][: t + 1], axis=0)), "err step %d" % t


@pytest.mark.parametrize("EW", [1, 2, 4, 8])  # EW 8: 12 cells x 8 envs > 64 lanes -> the list-based scan
def test_emu_robocup_trace(emu_lib, EW):
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "robocup_trace.npz"))
    run_trace(emu, lib, P.robocup_bodies(), None, tr, 1 | 4 | 16, EW, False)


@pytest.mark.parametrize("bp", [0, 32], ids=["full", "broadphase"])
@pytest.mark.parametrize("EW", [1, 2, 4])
def test_emu_lunar_trace(emu_lib, EW, bp):
    """bp = 32: COTIX_STAGE_BROADPHASE (separated polygon pairs skip GJK/EPA),
    the same golden trace bit for bit, choices included."""
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    rows = []
    for k in tr["terrain_keys"]:
        _, g = emu.oracle_scene(lib, P.lunar_lander_bodies(k))
        rows.append(g)
    run_trace(emu, lib, P.lunar_lander_bodies(tr["terrain_keys"][0]), rows, tr, 1 | 2 | 4 | 8 | 16 | bp, EW, True)


@pytest.mark.parametrize("EW", [2, 4, 8])
def test_emu_box_world_trace(emu_lib, EW):
    """The box world's 24 cells: 48 (cell, env) items at 2 envs per wave (one
    per lane), 96 at 4 (two per lane: the fused scan's second owner slot and
    its rank > 64 rounds), 192 at 8 (the list-compaction scan)."""
    emu, lib = emu_lib
    import make_golden as mg
    tr = np.load(os.path.join(GOLD, "box_world_trace.npz"))
    for e in range(tr["dyn"].shape[1]):
        sub = {k: tr[k][:, e:e + 1] for k in ("dyn", "keys", "err", "chosen", "cells")}
        run_trace(emu, lib, mg.box_world_bodies(e), None, sub, 1 | 4 | 16, EW, False)


def test_emu_order_clockwise_ties_nan_zero(emu_lib):
    """Stable order by angle (the kernel's rank sort) == the oracle's
    insertion sort, on duplicate vertices (ties), NaN coordinates and
    vertices whose angle is +-0 / +-pi."""
    emu, lib = emu_lib
    from cotix_oracle import geometry as G
    rng = np.random.default_rng(4)
    cases = []
    for nv in (3, 4, 6, 8):
        for _ in range(200):
            xy = rng.integers(-2, 3, size=(nv, 2)).astype(np.float32)  # many duplicates / collinear
            if rng.random() < 0.2:
                xy[rng.integers(nv), rng.integers(2)] = np.nan
            if rng.random() < 0.2:
                xy[rng.integers(nv)] = (-0.0, 0.0)
            cases.append(xy)
    for xy in cases:
        nv = xy.shape[0]
        got = np.ascontiguousarray(xy.reshape(-1).copy())
        lib.emu_order_clockwise(got.ctypes.data_as(emu.P_), 1, nv)
        want = np.array(G.order_clockwise([tuple(v) for v in xy]), np.float32).reshape(-1)
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (xy, got.reshape(-1, 2), want.reshape(-1, 2))


@pytest.mark.parametrize("EW", [1, 4])
@pytest.mark.parametrize("scenario", ["robocup", "lunar"])
def test_emu_fused_equals_single_steps(emu_lib, EW, scenario):
    """One launch of 37 fused steps (three key windows, the last one partial)
    == 37 one-step launches, bit for bit, with episode restarts on (RoboCup)."""
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    name = "robocup_trace.npz" if scenario == "robocup" else "lunar_trace.npz"
    tr = np.load(os.path.join(GOLD, name))
    if scenario == "robocup":
        h, geom = emu.oracle_scene(lib, P.robocup_bodies())
        gstride, stages = 0, 1 | 4 | 16
    else:
        rows = [emu.oracle_scene(lib, P.lunar_lander_bodies(k))[1] for k in tr["terrain_keys"]]
        h, _ = emu.oracle_scene(lib, P.lunar_lander_bodies(tr["terrain_keys"][0]))
        geom = np.ascontiguousarray(np.stack(rows).astype(np.float32))
        gstride, stages = geom.shape[1], 1 | 2 | 4 | 8 | 16 | 32
    dyn0 = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys0 = np.ascontiguousarray(tr["keys"][0]).astype(np.uint32)
    reset = dyn0.copy() if scenario == "robocup" else None
    B, T = dyn0.shape[2], 37
    fused = [dyn0.copy(), keys0.copy(), np.zeros(B, np.uint32)]
    emu.step(lib, h, *fused, geom, gstride, T, stages, E=EW, dyn_reset=reset)
    single = [dyn0.copy(), keys0.copy(), np.zeros(B, np.uint32)]
    for _ in range(T):
        emu.step(lib, h, *single, geom, gstride, 1, stages, E=EW, dyn_reset=reset)
    assert same_f32(fused[0], single[0])
    assert np.array_equal(fused[1], single[1]) and np.array_equal(fused[2], single[2])


def test_emu_robocup_autoreset_vs_cport(emu_lib):
    """Episode restarts (the bench workload) on CPU: the kernel logic vs the
    C port of the oracle, 64 perturbed envs x 2 launches of 20 fused steps."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    _build_cport()
    clib = cport.load()
    dyn, keys = cport.robocup_batch(64)
    dyn, keys = np.ascontiguousarray(dyn, np.float32), np.ascontiguousarray(keys, np.uint32)
    reset = dyn.copy()
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    sc = cport.Scene(clib, P.robocup_bodies())
    got = [dyn.copy(), keys.copy(), np.zeros(64, np.uint32), np.zeros(64, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(64, np.uint32), np.zeros(64, np.uint32)]
    for _ in range(2):
        emu.step(lib, h, got[0], got[1], got[2], geom, 0, 20, 1 | 4 | 16, E=4, dyn_reset=reset, resets=got[3])
        sc.step(want[0], want[1], want[2], 20, cport.STAGES_ROBOCUP, None, reset, want[3])
    assert want[3].sum() > 0
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("T", [64, 40, 33])
def test_emu_key_helper_vs_cport(emu_lib, T):
    """The step program with the key-window helper (cxk::KeyHelper: windows
    1.. computed by a helper wave into two alternating buffers, here at the
    step wave's barrier) on RoboCup with autoreset, actions and the collider
    trace == the C port -- and == the step without the helper, trace
    included.  T: 4 whole windows; a partial last window; a last window of one
    step (the helper's K0-K2 for n = 1 in place of k_one_regs)."""
    import ctypes
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    _build_cport()
    clib = cport.load()
    lib.emu_set_key_helper.argtypes = [ctypes.c_int]
    B = 12
    dyn, keys = cport.robocup_batch(B)
    dyn, keys = np.ascontiguousarray(dyn, np.float32), np.ascontiguousarray(keys, np.uint32)
    reset = dyn.copy()
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    sc = cport.Scene(clib, P.robocup_bodies())
    act = np.ascontiguousarray((np.random.default_rng(T).normal(size=(T, B, 2)) * 0.1).astype(np.float32))
    runs = []
    for helper in (1, 0):
        got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32), np.zeros(B, np.uint32)]
        try:
            lib.emu_set_key_helper(helper)
            tr = emu.step_ex(lib, h, got[0], got[1], got[2], geom, 0, T, 1 | 4 | 16, 5, E=4, action=act,
                             action_body=4, dyn_reset=reset, resets=got[3])
        finally:
            lib.emu_set_key_helper(0)
        runs.append((got, tr))
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32), np.zeros(B, np.uint32)]
    wch, wcl = sc.step_ex(want[0], want[1], want[2], T, cport.STAGES_ROBOCUP, None, act, 4, reset, want[3],
                          trace=True)
    (got, (gch, gcl)), (plain, (pch, pcl)) = runs
    assert want[3].sum() > 0
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert np.array_equal(got[0].view(np.uint32), plain[0].view(np.uint32))
    assert np.array_equal(gch, pch) and np.array_equal(gcl, pcl)


@pytest.mark.parametrize("EW", [2, 4, 8])
def test_emu_trace_actions_autoreset_vs_cport(emu_lib, EW):
    """cotix_step_ex on CPU: actions + episode restarts + the collider trace
    (chosen partner per body, winning candidate per cell) of the kernel logic
    == the C port, 96 perturbed RoboCup envs x 2 launches of 18 fused steps."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    _build_cport()
    clib = cport.load()
    B, T = 96, 18
    dyn, keys = cport.robocup_batch(B)
    dyn, keys = np.ascontiguousarray(dyn, np.float32), np.ascontiguousarray(keys, np.uint32)
    reset = dyn.copy()
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    sc = cport.Scene(clib, P.robocup_bodies())
    rng = np.random.default_rng(EW)
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32), np.zeros(B, np.uint32)]
    for _ in range(2):
        act = np.ascontiguousarray((rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32))
        gch, gcl = emu.step_ex(lib, h, got[0], got[1], got[2], geom, 0, T, 1 | 4 | 16, 5, E=EW, action=act,
                               action_body=4, dyn_reset=reset, resets=got[3])
        wch, wcl = sc.step_ex(want[0], want[1], want[2], T, cport.STAGES_ROBOCUP, None, act, 4, reset, want[3],
                              trace=True)
        assert np.array_equal(gch, wch)
        assert np.array_equal(gcl, wcl)
    assert want[3].sum() > 0 and (wcl >= 0).any()
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("bp", [0, 32], ids=["full", "broadphase"])
def test_emu_lunar_trace_vs_cport(emu_lib, bp):
    """LunarLander (GJK/EPA contacts) collider trace of the kernel logic == the
    C port: 24 envs with terrain per env, half of them dropped onto the ground;
    bp = 32 with the polygon broadphase (the C port has none)."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    _build_cport()
    clib = cport.load()
    B, T = 24, 10
    tk = prng.split(prng.PRNGKey(0), B)
    rows = np.ascontiguousarray(np.stack([emu.oracle_scene(lib, P.lunar_lander_bodies(k))[1] for k in tk]))
    h, _ = emu.oracle_scene(lib, P.lunar_lander_bodies(tk[0]))
    sc = cport.Scene(clib, P.lunar_lander_bodies(tk[0]))
    base = np.array([b.dyn() for b in P.lunar_lander_bodies(tk[0])], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[:3, 1, ::2] -= np.float32(6.3)
    dyn[:3, 3, ::2] = np.float32(-0.3)
    keys = np.ascontiguousarray(prng.split(prng.PRNGKey(1), B)).astype(np.uint32)
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    gch, gcl = emu.step_ex(lib, h, *got, rows, rows.shape[1], T, cport.STAGES_LUNAR | bp, 4, E=4)
    wch, wcl = sc.step_ex(*want, T, cport.STAGES_LUNAR, rows, trace=True)
    assert (wcl >= 0).sum() > B  # contacts were found
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])


def test_perfect_vertex_threshold():
    """circle_vs_aabb's `norm(v - ccp) < 1e-6` (cotix/_contacts.py:118) is
    evaluated in the kernels as `sumsq < 0x2b8cbccb` (no sqrt): with a
    correctly rounded sqrt the two agree for every float32 sum of squares."""
    T = np.uint32(0x2B8CBCCB).view(np.float32)
    c = np.float32(1e-6)
    bits = np.arange(0x2B8CBCCB - (1 << 20), 0x2B8CBCCB + (1 << 20), dtype=np.uint32)
    rng = np.random.default_rng(0)
    bits = np.concatenate([bits, rng.integers(0, 0x7F800001, 1 << 20, dtype=np.uint32),
                           np.array([0, 0x7F800000, 0x7FC00000], np.uint32)])
    s = bits.view(np.float32)
    assert np.array_equal(np.sqrt(s) < c, s < T)


@pytest.mark.parametrize("name", ["aabb_aabb", "circle_circle", "circle_aabb", "poly_poly", "aabb_poly",
                                  "circle_poly"])
def test_emu_contact_operators_vs_golden(emu_lib, name):
    """The kernels' contact functions (cotix_device.h, host build) on the
    ~6,000 golden operator cases, bit for bit, error bits included."""
    emu, lib = emu_lib
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a = np.ascontiguousarray(g[name + "_a"], np.float32)
    b = np.ascontiguousarray(g[name + "_b"], np.float32)
    n = a.shape[0]
    out = np.zeros((n, 4), np.float32)
    err = np.zeros(n, np.uint32)
    lib.emu_contacts(int(g[name + "_fn"]), n, a.ctypes.data_as(emu.P_), b.ctypes.data_as(emu.P_),
                     out.ctypes.data_as(emu.P_), err.ctypes.data_as(emu.P_))
    assert same_f32(out, g[name + "_out"])
    assert np.array_equal(err, g[name + "_err"])


def _edge_floats(rng, n):
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1e-38, np.pi, -np.pi, np.pi / 2,
                        -np.pi / 2, np.pi / 4, 3 * np.pi / 4, 1e4, -1e4, 0.41421356, 0.41421357, 1.0, -1.0],
                       np.float32)
    return np.concatenate([special, rng.normal(0, 3, n).astype(np.float32),
                           rng.uniform(-1e3, 1e3, n).astype(np.float32)])


def test_emu_transcendentals_vs_oracle(emu_lib):
    """sincos32 / atan2_32 of the kernels (cotix_device.h, branch-free selects)
    == the oracle's (branchy) restatement, bit for bit, on edge cases
    (+-0, +-inf, NaN, quadrant and octant boundaries) and random values."""
    emu, lib = emu_lib
    from cotix_oracle import geometry as G
    rng = np.random.default_rng(7)
    x = np.ascontiguousarray(_edge_floats(rng, 2000))
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    lib.emu_sincos(x.ctypes.data_as(emu.P_), x.size, s.ctypes.data_as(emu.P_), c.ctypes.data_as(emu.P_))
    want = np.array([G.sincos32(v) for v in x], np.float32)
    assert same_f32(s, want[:, 0]) and same_f32(c, want[:, 1])
    yy, xx = np.meshgrid(_edge_floats(rng, 60), _edge_floats(rng, 60))
    yy, xx = np.ascontiguousarray(yy.ravel()), np.ascontiguousarray(xx.ravel())
    out = np.zeros_like(yy)
    lib.emu_atan2(yy.ctypes.data_as(emu.P_), xx.ctypes.data_as(emu.P_), yy.size, out.ctypes.data_as(emu.P_))
    want = np.array([G.atan2_32(a, b) for a, b in zip(yy, xx)], np.float32)
    assert same_f32(out, want)


@pytest.mark.parametrize("bp", [0, 32], ids=["full", "broadphase"])
@pytest.mark.parametrize("EW", [1, 4, 8])
def test_emu_lunar_restarts_move_static_body_vs_cport(emu_lib, EW, bp):
    """Phase T keeps a body's world parts while its pose bits are unchanged
    (the static terrain): restarts into a reset state whose terrain body sits
    elsewhere (and a NaN-posed lander in some envs) must rebuild them.  The
    kernel logic == the C port over 2 launches of 9 fused steps; envs with an
    error bit at launch start restart after their first step."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    _build_cport()
    clib = cport.load()
    B, T = 20, 9
    tk = prng.split(prng.PRNGKey(4), B)
    rows = np.ascontiguousarray(np.stack([emu.oracle_scene(lib, P.lunar_lander_bodies(k))[1] for k in tk]))
    h, _ = emu.oracle_scene(lib, P.lunar_lander_bodies(tk[0]))
    sc = cport.Scene(clib, P.lunar_lander_bodies(tk[0]))
    base = np.array([b.dyn() for b in P.lunar_lander_bodies(tk[0])], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[:3, 1, :] -= np.float32(6.3)  # dropped onto the terrain
    dyn[:3, 3, :] = np.float32(-0.3)
    reset = dyn.copy()
    reset[3, 0, 0::2] += np.float32(0.75)  # the terrain body restarts elsewhere
    reset[3, 4, 1::2] = np.float32(2.0)    # ... or only rotated (vertex order changes)
    reset[0, 4, 3::5] = np.float32(np.nan)  # a NaN-posed lander
    keys = np.ascontiguousarray(prng.split(prng.PRNGKey(5), B)).astype(np.uint32)
    err0 = np.zeros(B, np.uint32)
    err0[1::3] = 1
    got = [dyn.copy(), keys.copy(), err0.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), err0.copy(), np.zeros(B, np.uint32)]
    for launch in range(2):
        gch, gcl = emu.step_ex(lib, h, got[0], got[1], got[2], rows, rows.shape[1], T, cport.STAGES_LUNAR | bp, 4,
                               E=EW, dyn_reset=reset, resets=got[3])
        wch, wcl = sc.step_ex(want[0], want[1], want[2], T, cport.STAGES_LUNAR, rows, None, 0, reset, want[3],
                              trace=True)
        assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
        if launch == 0:
            got[2][0::4] = 1
            want[2][0::4] = 1
    assert want[3].sum() == len(err0[1::3]) + len(err0[0::4])
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


def test_reference_scenes_get_their_specializations(emu_lib):
    """The two reference scenes, under the default constants in either PRNG
    layout, compile to the constant headers of their step-kernel
    specializations (cxk::SPEC_HDRS): a scene-compiler change that moved them
    would silently fall back to the generic kernel.  Any other constant set
    runs the generic kernel."""
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    from cotix_oracle.params import Params
    lib.emu_scene_spec.argtypes = [ctypes.c_void_p]
    for bodies, spec in ((P.robocup_bodies, 1), (P.lunar_lander_bodies, 2)):
        h, _ = emu.oracle_scene(lib, bodies())
        assert lib.emu_scene_spec(h) == spec
        h, _ = emu.oracle_scene(lib, bodies(), Params(prng_layout="partitionable"))
        assert lib.emu_scene_spec(h) == spec + 2
        for alt in (dict(contact_p=0.3), dict(gjk_max_steps=31), dict(baumgarte=0.2),
                    dict(prng_layout="partitionable", epa_max_iters=47)):
            h, _ = emu.oracle_scene(lib, bodies(), Params(**alt))
            assert lib.emu_scene_spec(h) == 0, alt
    # the box world's structure (any parameter values of 3 AABB walls + 4 circles)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_spec_hdrs
    h, _ = emu.oracle_scene(lib, gen_spec_hdrs.box_bodies())
    assert lib.emu_scene_spec(h) == 5
    h, _ = emu.oracle_scene(lib, gen_spec_hdrs.box_bodies(), Params(prng_layout="partitionable"))
    assert lib.emu_scene_spec(h) == 0


def test_specialization_headers_are_current():
    """parallax_amd/csrc/cotix_spec_hdrs.h is what tools/gen_spec_hdrs.py
    writes from the current scene compiler (the kernel folds these headers)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_spec_hdrs.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_reference_scenes_fit_the_lds(emu_lib):
    """The step kernel's workgroup LDS (hot tables + 4 wave tiles + scratch)
    stays within the CU's 160 KiB for the tilings the library launches: every
    envs-per-wave for RoboCup, 1/2/4 for LunarLander (the default is 4)."""
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    lib.emu_lds_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.emu_lds_bytes.restype = ctypes.c_long
    h, _ = emu.oracle_scene(lib, P.robocup_bodies())
    assert all(lib.emu_lds_bytes(h, e) <= 160 * 1024 for e in (1, 2, 4, 8))
    h, _ = emu.oracle_scene(lib, P.lunar_lander_bodies())
    assert all(lib.emu_lds_bytes(h, e) <= 160 * 1024 for e in (1, 2, 4))


@pytest.mark.parametrize("bp", [0, 32], ids=["full", "broadphase"])
@pytest.mark.parametrize("EW", [1, 2, 4])
def test_emu_static_part_straddling_chunks_vs_cport(emu_lib, EW, bp):
    """Phase T with a kept (static) body whose part straddles two vertex-item
    chunks, the first of which runs for the moving body: the straddling part
    must be kept whole (rebuilding half of it would read the other half's dead
    vertex items).  The kernel logic == the C port over 20 steps, 6 envs."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    _build_cport()
    clib = cport.load()
    import scene_cases
    bodies = scene_cases.straddle_scene(4.0)
    h, geom = emu.oracle_scene(lib, bodies)
    sc = cport.Scene(clib, bodies)
    B, T = 6, 20
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[0, 0, :] += np.linspace(-1, 1, B).astype(np.float32)
    keys = np.ascontiguousarray(np.stack([np.arange(B), np.arange(B) * 7 + 1], 1).astype(np.uint32))
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    gch, gcl = emu.step_ex(lib, h, *got, geom, 0, T, 1 | 4 | 16 | bp, 2, E=EW)
    wch, wcl = sc.step_ex(*want, T, 1 | 4 | 16, trace=True)
    assert (wcl[:, 0, 1] >= 0).sum() + (wcl[:, 1, 0] >= 0).sum() > T  # the triangle sits on the floor
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


def test_emu_octagon_row_one_env_per_wave_vs_cport(emu_lib):
    """A scene whose tile fits the LDS at one env per wave only (9 octagon
    bodies, scene_cases.octagon_row; the library picks that tiling at
    cotix_scene_create): the kernel logic at EW 1 == the C port over 16 steps,
    4 envs, contact choices included."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    _build_cport()
    clib = cport.load()
    import scene_cases
    bodies = scene_cases.octagon_row(9)
    h, geom = emu.oracle_scene(lib, bodies)
    lib.emu_lds_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.emu_lds_bytes.restype = ctypes.c_long
    assert lib.emu_lds_bytes(h, 1) <= 160 * 1024 < lib.emu_lds_bytes(h, 2)
    sc = cport.Scene(clib, bodies)
    B, T = 4, 16
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[1:, 2, :] += np.linspace(-0.2, 0.2, B).astype(np.float32)
    keys = np.ascontiguousarray(np.stack([np.arange(B) + 9, np.arange(B) * 3 + 2], 1).astype(np.uint32))
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    gch, gcl = emu.step_ex(lib, h, *got, geom, 0, T, 1 | 4 | 16, len(bodies), E=1)
    wch, wcl = sc.step_ex(*want, T, 1 | 4 | 16, trace=True)
    assert (wcl >= 0).sum() > 4 * T  # neighbours in contact
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("name", ["octagons12", "octagons15", "polygon20"])
def test_emu_large_scenes_vs_cport(emu_lib, name):
    """Scenes whose tiles fit the LDS only in workgroups of fewer than four
    waves (cotix_scene_waves_per_group): twelve and fifteen octagon bodies,
    and 20 polygon parts over 5 bodies -- the kernel logic at one env per
    wave == the C port over 12 steps, 3 envs, the collider trace included."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    _build_cport()
    clib = cport.load()
    import scene_cases
    bodies = scene_cases.polygon20() if name == "polygon20" else scene_cases.octagon_row(int(name[8:]))
    h, geom = emu.oracle_scene(lib, bodies)
    lib.emu_lds_bytes_w.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.emu_lds_bytes_w.restype = ctypes.c_long
    assert lib.emu_lds_bytes_w(h, 1, 4) > 160 * 1024 >= lib.emu_lds_bytes_w(h, 1, 1)
    sc = cport.Scene(clib, bodies)
    B, T = 3, 12
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[1:, 2, :] += np.linspace(-0.2, 0.2, B).astype(np.float32)
    keys = np.ascontiguousarray(np.stack([np.arange(B) + 9, np.arange(B) * 3 + 2], 1).astype(np.uint32))
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    gch, gcl = emu.step_ex(lib, h, *got, geom, 0, T, 1 | 4 | 16, len(bodies), E=1)
    wch, wcl = sc.step_ex(*want, T, 1 | 4 | 16, trace=True)
    assert (wcl >= 0).sum() > B * T  # contacts written
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("EW", [1, 4, 8])
def test_emu_robocup_moving_static_bodies_vs_cport(emu_lib, EW):
    """The analytic program with infinite-mass bodies that do move: restarts
    into a reset state whose goal body sits elsewhere, a NaN-posed play area,
    an infinite-mass goal that moves every step in half of the envs and an
    AABB body whose angle alone changes.  The kernel logic == the C port
    (trace of the chosen partners and winning candidates too) over 2 launches
    of 9 fused steps; envs with an error bit at launch start restart after
    their first step."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    _build_cport()
    clib = cport.load()
    B, T = 20, 9
    dyn, keys = cport.robocup_batch(B)
    dyn, keys = np.ascontiguousarray(dyn, np.float32), np.ascontiguousarray(keys, np.uint32)
    dyn[2, 2, 0::2] = np.float32(0.5)  # a moving infinite-mass goal
    dyn[3, 5, 1::4] = np.float32(3.0)  # a spinning AABB body: same world words every step
    reset = dyn.copy()
    reset[2, 0, 1::2] += np.float32(0.75)  # the goal restarts elsewhere
    reset[1, 1, 3::5] = np.float32(np.nan)  # a NaN-posed play area
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    sc = cport.Scene(clib, P.robocup_bodies())
    err0 = np.zeros(B, np.uint32)
    err0[1::3] = 1
    got = [dyn.copy(), keys.copy(), err0.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), err0.copy(), np.zeros(B, np.uint32)]
    for launch in range(2):
        gch, gcl = emu.step_ex(lib, h, got[0], got[1], got[2], geom, 0, T, cport.STAGES_ROBOCUP, 5, E=EW,
                               dyn_reset=reset, resets=got[3])
        wch, wcl = sc.step_ex(want[0], want[1], want[2], T, cport.STAGES_ROBOCUP, None, None, 0, reset, want[3],
                              trace=True)
        assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
        if launch == 0:
            got[2][0::4] = 1
            want[2][0::4] = 1
    assert want[3].sum() >= len(err0[1::3]) + len(err0[0::4])
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("circle", [False, True], ids=["aabb_poly", "aabb_circle_poly"])
@pytest.mark.parametrize("EW", [2, 4])
def test_emu_mixed_kinds_step_vs_cport(emu_lib, EW, circle):
    """The step kernel's AABB x polygon (and circle x polygon) programs
    (cxk::launch_fnset 11 / 15): two quads falling onto a static AABB floor
    (one in contact with the other), optionally a ball; the kernel logic == the
    C port over 20 steps, 6 envs."""
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    _build_cport()
    clib = cport.load()
    quad = [(-0.5, 0.0), (0.5, 0.0), (0.5, 0.6), (-0.5, 0.6)]
    bodies = [P.Body([G.Polygon(quad, kind="Polygon4")], position=(0.1, 0.02), velocity=(0.0, -0.4),
                     angular_velocity=0.2, elasticity=0.5, friction_coefficient=0.2),
              P.Body([G.Polygon(quad, kind="Polygon4")], position=(0.95, 0.3), angle=0.3, velocity=(-0.2, -0.3),
                     elasticity=0.5, friction_coefficient=0.2),
              P.Body([G.AABB((-4.0, -1.0), (4.0, 0.0))], mass=float("inf"), inertia=float("inf"), elasticity=0.5,
                     friction_coefficient=0.2)]
    if circle:
        bodies.insert(2, P.Body([G.Circle(0.3, (0.0, 0.0))], position=(-0.75, 0.25), velocity=(0.3, -0.2),
                                elasticity=0.5, friction_coefficient=0.2))
    h, geom = emu.oracle_scene(lib, bodies)
    sc = cport.Scene(clib, bodies)
    B, T = 6, 20
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[0, 0, :] += np.linspace(-0.3, 0.3, B).astype(np.float32)
    keys = np.ascontiguousarray(np.stack([np.arange(B) + 3, np.arange(B) * 5 + 1], 1).astype(np.uint32))
    got = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    nb = len(bodies)
    gch, gcl = emu.step_ex(lib, h, *got, geom, 0, T, 1 | 4 | 16, nb, E=EW)
    wch, wcl = sc.step_ex(*want, T, 1 | 4 | 16, trace=True)
    assert (wcl >= 0).sum() > T  # contacts were found
    assert np.array_equal(gch, wch) and np.array_equal(gcl, wcl)
    assert same_f32(got[0], want[0])
    for g, w in zip(got[1:], want[1:]):
        assert np.array_equal(g, w)


def test_scan_items_past_the_last_rank(emu_lib):
    """The fused scan draws for at most COTIX_SCAN_RANKS pending items per
    round (64 in the library); the others wait for a later round.  A build
    with 3 ranks runs that path on every step: the traces stay bit-exact
    (RoboCup at 4 and 8 envs per wave -- one and two items per lane --, the
    box world at 4, LunarLander at 4)."""
    import ctypes
    emu, real = emu_lib
    out = os.path.join(HERE, "emu", "build", "libcotix_emu_ranks3.so")
    src = os.path.join(HERE, "emu", "cotix_emu.cpp")
    deps = [src] + [os.path.join(ROOT, "parallax_amd", "csrc", f) for f in os.listdir(
        os.path.join(ROOT, "parallax_amd", "csrc")) if f.endswith(".h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(f) for f in deps):
        tmp = "%s.%d.tmp" % (out, os.getpid())
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-w",
                        "-DCOTIX_SCAN_RANKS=3", src, "-o", tmp], check=True)
        os.replace(tmp, out)
    lib = ctypes.CDLL(out)
    for fn in ("emu_scene_create", "emu_scene_create_ex", "emu_step", "emu_step_ex"):
        getattr(lib, fn).argtypes = getattr(real, fn).argtypes
    lib.emu_last_error.restype = ctypes.c_char_p
    from cotix_oracle import physics as P
    import make_golden as mg
    tr = np.load(os.path.join(GOLD, "robocup_trace.npz"))
    for EW in (4, 8):
        run_trace(emu, lib, P.robocup_bodies(), None, tr, 1 | 4 | 16, EW, False)
    tb = np.load(os.path.join(GOLD, "box_world_trace.npz"))
    for e in range(tb["dyn"].shape[1]):
        sub = {k: tb[k][:, e:e + 1] for k in ("dyn", "keys", "err", "chosen", "cells")}
        run_trace(emu, lib, mg.box_world_bodies(e), None, sub, 1 | 4 | 16, 4, False)
    tl = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    rows = [emu.oracle_scene(real, P.lunar_lander_bodies(k))[1] for k in tl["terrain_keys"]]
    run_trace(emu, lib, P.lunar_lander_bodies(tl["terrain_keys"][0]), rows, tl, 1 | 2 | 4 | 8 | 16, 4, True)
