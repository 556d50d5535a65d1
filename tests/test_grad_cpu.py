"""Differentiable rollout (BASELINE config 5) on CPU: the kernel's forward
and backward wave programs (host emulation, tests/emu) against the torch
float32 VJP chain of the oracle (oracle/cotix_oracle/grad.py), itself
checked against central finite differences of the faithful oracle."""
import os
import sys

import numpy as np
import pytest

import grad_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emu_lib():
    import subprocess
    import sys
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    return emu, emu.load()


def _both_backwards(emu, lib, h, sd, sk, tape, geom, stages, case, E):
    """The tape backward (MODE 4, what the library runs) and the re-play
    (MODE 2): bit for bit the same gradients, NaN patterns included."""
    args = (geom, 0, stages, case["actions"], case["ab"], case["w"])
    ga, gd = emu.rollout_backward(lib, h, sd, sk, *args, E=E, tape=tape)
    ra, rd = emu.rollout_backward(lib, h, sd, sk, *args, E=E)
    assert np.array_equal(ga.view(np.uint32), ra.view(np.uint32)), "grad_action: tape != re-play"
    assert np.array_equal(gd.view(np.uint32), rd.view(np.uint32)), "grad_dyn0: tape != re-play"
    return ga, gd


def _emu_run(emu, lib, case, E=4):
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    keys = np.array(case["keys"], np.uint32, copy=True)  # the kernel advances keys in place
    err = np.zeros(dyn.shape[2], np.uint32)
    ret, sd, sk, tape = emu.rollout(lib, h, dyn, keys, err, geom, 0, 1 | 4 | 16, case["actions"], case["ab"],
                                    case["w"], E=E)
    ga, gd = _both_backwards(emu, lib, h, sd, sk, tape, geom, 1 | 4 | 16, case, E)
    return ret, ga, gd, dyn


@pytest.mark.parametrize("E", [4, 1])
def test_saved_rows_env_blocks(emu_lib, E):
    """The forward saves the state before step t in env blocks of 4
    (cxk::row_at); parallax_amd.trajectory unpacks them: equal to the state
    after a t-step rollout, for a batch that is not a multiple of 4."""
    import torch
    from parallax_amd.rollout import trajectory
    emu, lib = emu_lib
    case = GC.box_case(5, 6, seed=11)
    T = case["actions"].shape[0]
    h, geom = emu.oracle_scene(lib, case["make"]())

    def run(n):
        dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
        keys = np.array(case["keys"], np.uint32, copy=True)
        err = np.zeros(dyn.shape[2], np.uint32)
        out = emu.rollout(lib, h, dyn, keys, err, geom, 0, 1 | 4 | 16, case["actions"][:n], case["ab"], case["w"],
                          E=E)
        return dyn, out[1]

    _, sd = run(T)
    assert sd.shape == (T, 2, dyn_words(case), 4)
    traj = trajectory({"dyn": torch.from_numpy(sd)}, 5).numpy()
    for t in range(T):
        want = run(t)[0] if t > 0 else np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
        assert np.array_equal(traj[t].view(np.uint32), want.view(np.uint32)), t


def dyn_words(case):
    return case["S0"].shape[1] * 6


def test_oracle_grad_vs_finite_differences():
    """The checker itself: torch VJP chain vs central differences of the
    faithful f32 oracle (box world, no discrete flips at eps=1e-2)."""
    case = GC.box_case(2, 10, seed=3)
    orc = GC.oracle(case)
    P = GC.P
    for e in range(2):
        ga = orc[e][1]
        for (t, c) in [(0, 0), (0, 1), (4, 0), (9, 1)]:
            vals = []
            for s in (1, -1):
                a = case["actions"][:, e].copy()
                a[t, c] += s * 1e-2
                bodies = case["make"]()
                for b, row in zip(bodies, case["S0"][e]):
                    b.set_dyn(row)
                key = case["keys"][e]
                tot = 0.0
                for tt in range(10):
                    bodies, key = P.robocup_step(bodies, key, GC.D0, action=a[tt], action_body=case["ab"])
                    tot += float(bodies[6].position[0]) + 0.5 * float(bodies[5].velocity[1])
                vals.append(tot)
            fd = (vals[0] - vals[1]) / 2e-2
            assert abs(fd - ga[t, c]) <= 2e-3 * (1 + abs(fd)), (e, t, c, fd, ga[t, c])


# (T 32: the GPU test's horizon; B 8 at 4 envs per wave: the backward's
# 16-byte row restore, two steps ahead -- B 6 its one-word form)
@pytest.mark.parametrize("E,T,B", [(1, 40, 6), (4, 32, 6), (4, 32, 8)])
def test_emu_rollout_box_world(emu_lib, E, T, B):
    emu, lib = emu_lib
    case = GC.box_case(B, T, seed=1)
    ret, ga, gd, dyn = _emu_run(emu, lib, case, E)
    orc = GC.oracle(case)
    for e in range(B):
        r, oga, ogS = orc[e]
        assert np.float32(ret[e]).view(np.uint32) == np.float32(r).view(np.uint32), (e, ret[e], r)  # bit-exact
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d grad_action: %s" % (e, msg)
        ok, msg = GC.close(gd[:, :, e], ogS, case["tol"], case["name"])
        assert ok, "env %d grad_dyn0: %s" % (e, msg)
    assert np.abs(ga).max() > 0


def test_emu_rollout_robocup(emu_lib):
    """The config-5 scene itself (short horizon): ball x return, NaN-propagation
    pattern included (most RoboCup envs go NaN at step 1 in the reference)."""
    emu, lib = emu_lib
    B, T = 8, 6
    case = GC.robocup_case(B, T)
    ret, ga, gd, _ = _emu_run(emu, lib, case)
    orc = GC.oracle(case)
    finite = 0
    for e in range(B):
        r, oga, ogS = orc[e]
        same = (np.isnan(ret[e]) and np.isnan(r)) or np.float32(ret[e]).view(np.uint32) == np.float32(r).view(
            np.uint32)
        assert same, (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d: %s" % (e, msg)
        finite += int(np.isfinite(oga).all())
    assert finite >= 1


LUNAR_STAGES = 1 | 2 | 4 | 8 | 16 | 32  # incl. the broadphase (the backward re-plays without it)


def _fd_actions(case, e, points, eps=1e-2):
    """Central differences of the faithful oracle's return in the actions."""
    T = case["actions"].shape[0]
    out = []
    for (t, c) in points:
        vals = []
        for s in (1, -1):
            a = case["actions"][:, e].copy()
            a[t, c] += s * eps
            bodies = case["make"]()
            for b, row in zip(bodies, case["S0"][e]):
                b.set_dyn(row)
            key, tot = case["keys"][e], 0.0
            for tt in range(T):
                bodies, key = case["step"](bodies, key, GC.D0, action=a[tt], action_body=case["ab"])
                tot += float(np.dot(case["w"], np.array([b.dyn() for b in bodies], np.float64).reshape(-1)))
            vals.append(tot)
        out.append((vals[0] - vals[1]) / (2 * eps))
    return out


@pytest.mark.parametrize("scene", ["lunar", "poly_box", "ball_poly"])
def test_oracle_grad_polygons_vs_finite_differences(scene, monkeypatch):
    """The checker through GJK/EPA, contact_from_edges and (LunarLander) the
    joints, and (ball_poly) circle x polygon's GJK + EPA with the circle's
    direction-dependent support: torch VJP chain vs central differences of
    the faithful oracle (cases without discrete flips at eps = 1e-2)."""
    case = {"lunar": lambda: GC.lunar_case(4, 6, seed=0), "poly_box": lambda: GC.poly_box_case(4, 10, seed=0),
            "ball_poly": lambda: GC.ball_poly_case(4, 10, seed=0)}[scene]()
    from cotix_oracle import grad as OG
    calls = []
    real = OG._circle_polygon_contact
    monkeypatch.setattr(OG, "_circle_polygon_contact", lambda *a: calls.append(1) or real(*a))
    orc = GC.oracle(case)
    assert (len(calls) > 10) == (scene == "ball_poly")  # circle x polygon resolutions differentiated
    pts = [(0, 0), (0, 1), (2, 0), (5, 1)]
    nontrivial = 0
    for e in range(4):
        ga = orc[e][1]
        for (t, c), fd in zip(pts, _fd_actions(case, e, pts)):
            assert abs(fd - ga[t, c]) <= 2e-3 * (1 + abs(fd)), (e, t, c, fd, ga[t, c])
            nontrivial += int(abs(ga[t, c]) > 1e-3)
    assert nontrivial >= 8


def _emu_run_st(emu, lib, case, stages, E=4, params=None):
    from cotix_oracle import params as _params
    with _params.use(params):  # (the scene's own draws, LunarLander's terrain, in the block's layout)
        bodies = case["make"]()
    h, geom = emu.oracle_scene(lib, bodies, params)
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    keys = np.array(case["keys"], np.uint32, copy=True)
    err = np.zeros(dyn.shape[2], np.uint32)
    ret, sd, sk, tape = emu.rollout(lib, h, dyn, keys, err, geom, 0, stages, case["actions"], case["ab"], case["w"],
                                    E=E)
    ga, gd = _both_backwards(emu, lib, h, sd, sk, tape, geom, stages, case, E)
    return ret, ga, gd


def _check_vs_oracle(case, ret, ga, gd, params=None):
    orc = GC.oracle(case, params=params)
    for e in orc:
        r, oga, ogS = orc[e]
        assert np.float32(ret[e]).view(np.uint32) == np.float32(r).view(np.uint32), (e, ret[e], r)  # bit-exact
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d grad_action: %s" % (e, msg)
        ok, msg = GC.close(gd[:, :, e], ogS, case["tol"], case["name"])
        assert ok, "env %d grad_dyn0: %s" % (e, msg)


@pytest.mark.parametrize("E", [1, 4])
def test_emu_rollout_lunar(emu_lib, E):
    """LunarLander with its legs on the pad: polygon x polygon contacts every
    step plus the four joints, 12 steps, against the VJP oracle."""
    emu, lib = emu_lib
    case = GC.lunar_case(4, 12, seed=0)
    ret, ga, gd = _emu_run_st(emu, lib, case, LUNAR_STAGES, E)
    _check_vs_oracle(case, ret, ga, gd)
    assert np.abs(gd[:, :, :]).max() > 1.0


@pytest.mark.parametrize("octagons", [False, True])
def test_emu_rollout_poly_box(emu_lib, octagons):
    """AABB x polygon and polygon x polygon contacts of two rotating polygons
    (octagons: the 80-term contact_from_edges pairs)."""
    emu, lib = emu_lib
    case = GC.poly_box_case(6, 10, seed=0, octagons=octagons)
    ret, ga, gd = _emu_run_st(emu, lib, case, 1 | 4 | 16)
    _check_vs_oracle(case, ret, ga, gd)


def test_emu_rollout_quad_row(emu_lib):
    """Nine polygons of one contact type: the contact VJPs inside phase G's
    chain (no room for phase GE's responses in the key window)."""
    emu, lib = emu_lib
    case = GC.quad_row_case(4, 6, seed=0)
    ret, ga, gd = _emu_run_st(emu, lib, case, 1 | 4 | 16)
    _check_vs_oracle(case, ret, ga, gd)


def test_backward_rejects_long_gjk_circle_polygon_and_analytic_joints(emu_lib):
    """Circle x polygon gradients record every GJK point: a parameter block
    with gjk_max_steps > 32 is refused for them; the joint stage needs the
    polygon program."""
    emu, lib = emu_lib
    from cotix_oracle import geometry as Gm
    from cotix_oracle import physics as P
    from cotix_oracle import params as OPr
    bodies = GC.poly_box_bodies() + [P.Body([Gm.Circle(0.2, (0.0, 0.0))], position=(1.5, 0.2))]
    h, geom = emu.oracle_scene(lib, bodies, OPr.Params(gjk_max_steps=33))
    sd = np.zeros((1, 5, 6, 1), np.float32)
    sk = np.zeros((1, 1, 2), np.uint32)
    with pytest.raises(RuntimeError, match="circle x polygon"):
        emu.rollout_backward(lib, h, sd, sk, geom, 0, 1 | 4 | 16, np.zeros((1, 1, 2), np.float32), 0,
                             np.zeros(30, np.float32))
    case = GC.box_case(1, 1)
    h, geom = emu.oracle_scene(lib, case["make"]())
    with pytest.raises(RuntimeError, match="joint stage"):
        emu.rollout_backward(lib, h, np.zeros((1, 7, 6, 1), np.float32), sk, geom, 0, 1 | 4 | 8 | 16,
                             np.zeros((1, 1, 2), np.float32), 0, np.zeros(42, np.float32))


@pytest.mark.parametrize("nterms", [8, 42])
def test_emu_rollout_return_terms(emu_lib, nterms):
    """The forward's return over more nonzero weights: 8 terms (the compact
    list's capacity) and all 42 (past it: the weights from the kernel
    arguments), bit-exact returns and the gradients vs the VJP oracle."""
    emu, lib = emu_lib
    B, T = 3, 8
    case = GC.box_case(B, T, seed=2)
    rng = np.random.default_rng(5)
    w = np.zeros(7 * 6, np.float32)
    idx = np.sort(rng.choice(42, nterms, replace=False))
    w[idx] = rng.uniform(-1, 1, nterms).astype(np.float32)
    case["w"] = w
    ret, ga, gd, _ = _emu_run(emu, lib, case)
    orc = GC.oracle(case)
    for e in range(B):
        r, oga, ogS = orc[e]
        assert np.float32(ret[e]).view(np.uint32) == np.float32(r).view(np.uint32), (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d grad_action: %s" % (e, msg)


@pytest.mark.parametrize("sfx", ["_part", "_alt"])
@pytest.mark.parametrize("scene", ["box", "lunar", "poly_box"])
def test_emu_rollout_under_param_sets(emu_lib, scene, sfx):
    """The differentiable rollout under a non-default parameter block
    (tests/param_sets.py: the partitionable PRNG layout; Baumgarte 0.2 / 0.02,
    bernoulli p 0.3, GJK capped at 1 step, EPA at 3 iterations): the backward
    reads the scene's Baumgarte constants, narrowphase caps and (re-play) PRNG
    layout -- emulation (tape == re-play) against the VJP oracle run under the
    same block, returns bit for bit."""
    from param_sets import oracle_params
    emu, lib = emu_lib
    prm = oracle_params(sfx)
    case, stages = {"box": (GC.box_case(4, 12, seed=4), 1 | 4 | 16),
                    "lunar": (GC.lunar_case(4, 8, seed=1), LUNAR_STAGES),
                    "poly_box": (GC.poly_box_case(4, 8, seed=2), 1 | 4 | 16)}[scene]
    ret, ga, gd = _emu_run_st(emu, lib, case, stages, params=prm)
    _check_vs_oracle(case, ret, ga, gd, params=prm)


def test_g_regs_equals_tile_form(emu_lib):
    """Phase G's register form for the analytic scenes (g_regs: RoboCup's 5
    and the box world's 7 bodies) against the tile form every other scene
    runs (a host build with -DCOTIX_NO_GREGS): the same gradients, NaN
    patterns included (NaN payloads aside -- the host's NaN sign follows the
    operand order of the two forms)."""
    import subprocess
    emu, lib = emu_lib
    d = os.path.join(HERE, "emu")
    out = os.path.join(d, "build", "libcotix_emu_nogregs.so")
    subprocess.run(["g++", "-O2", "-DCOTIX_EMU_POISON", "-DCOTIX_NO_GREGS", "-std=c++17", "-fPIC", "-shared",
                    "-ffp-contract=off", "-fno-fast-math", "-w", "cotix_emu.cpp", "-o", out], cwd=d, check=True)
    tile = emu.load(path=out)
    for case in (GC.box_case(6, 32, seed=1), GC.robocup_case(4, 20, seed=0)):
        ra, rb = _emu_run(emu, lib, case, 4), _emu_run(emu, tile, case, 4)
        for x, y in zip(ra[:3], rb[:3]):
            x, y = np.asarray(x, np.float32), np.asarray(y, np.float32)
            nx, ny = np.isnan(x), np.isnan(y)
            assert np.array_equal(nx, ny)
            assert np.array_equal(x[~nx].view(np.uint32), y[~ny].view(np.uint32))


@pytest.mark.parametrize("scene", ["box", "robocup"])
def test_split_backward_equals_tape_backward(emu_lib, scene):
    """The split tape backward (cxk::run_backward_split: a producer wave's
    restore / Euler / world parts / phase D of step s into one of two tiles
    while a consumer wave reverses step s + 1 on the other, adjoints in the
    consumer's registers) run on the emulation as producer-then-consumer per
    step: bit for bit the one-wave tape backward (MODE 4), NaN patterns
    included -- odd and even horizons (the two tiles' alternation), a batch
    whose last wave is partly idle."""
    import ctypes
    emu, lib = emu_lib
    lib.emu_set_split_bwd.argtypes = [ctypes.c_int]
    for T, B in ((7, 8), (8, 12)):
        case = GC.box_case(B, T, seed=5) if scene == "box" else GC.robocup_case(B, T, seed=2)
        h, geom = emu.oracle_scene(lib, case["make"]())
        dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
        keys = np.array(case["keys"], np.uint32, copy=True)
        err = np.zeros(dyn.shape[2], np.uint32)
        _, sd, sk, tape = emu.rollout(lib, h, dyn, keys, err, geom, 0, 1 | 4 | 16, case["actions"], case["ab"],
                                      case["w"], E=4)
        args = (geom, 0, 1 | 4 | 16, case["actions"], case["ab"], case["w"])
        try:
            lib.emu_set_split_bwd(1)
            sa, sg = emu.rollout_backward(lib, h, sd, sk, *args, E=4, tape=tape)
        finally:
            lib.emu_set_split_bwd(0)
        ta, tg = emu.rollout_backward(lib, h, sd, sk, *args, E=4, tape=tape)
        assert np.array_equal(sa.view(np.uint32), ta.view(np.uint32)), (scene, T, "grad_action")
        assert np.array_equal(sg.view(np.uint32), tg.view(np.uint32)), (scene, T, "grad_dyn0")
        assert np.isfinite(sa).any()


def test_circle_poly_recorded_forward_is_the_forward(emu_lib):
    """The circle x polygon gradient re-runs GJK + EPA while recording every
    Minkowski point (cx::cp_forward): its final edge gives the forward
    contact's penetration bit for bit (cx::circle_vs_polygon, 128 EPA
    iterations) over the golden circle x polygon pairs and random ones."""
    import ctypes
    emu, lib = emu_lib
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden as M
    from cotix_oracle import geometry as Gm
    rng = np.random.default_rng(5)
    pairs = [(Gm.Circle(np.float32(rng.uniform(0.2, 1.5)), (np.float32(rng.normal() * 0.7),
                                                             np.float32(rng.normal() * 0.7))),
              M.rand_poly(rng, n)) for n in (3, 4, 5, 6, 8) for _ in range(200)]
    a = np.ascontiguousarray(np.array([M.row(c) for c, _ in pairs], np.float32))
    b = np.ascontiguousarray(np.array([M.row(p) for _, p in pairs], np.float32))
    n = len(pairs)
    pf, pr = np.zeros((n, 2), np.float32), np.zeros((n, 2), np.float32)
    P_ = ctypes.c_void_p
    lib.emu_circle_poly_check(n, a.ctypes.data_as(P_), b.ctypes.data_as(P_), pf.ctypes.data_as(P_),
                              pr.ctypes.data_as(P_))
    hit = ~np.isnan(pr).any(1)
    assert hit.sum() > 200
    assert np.array_equal(pf[hit].view(np.uint32), pr[hit].view(np.uint32))


@pytest.mark.parametrize("E", [1, 4])
def test_emu_rollout_ball_on_polygons(emu_lib, E):
    """Gradients through circle x polygon contacts (GJK + EPA with the
    circle's direction-dependent support, every point of the chain): the
    kernel logic's tape backward and re-play agree bit for bit and match the
    torch-f32 VJP oracle (itself checked against finite differences above)."""
    emu, lib = emu_lib
    case = GC.ball_poly_case(8, 12, seed=1)
    ret, ga, gd = _emu_run_st(emu, lib, case, 1 | 4 | 16, E=E)
    from cotix_oracle import grad as OG
    calls = []
    real = OG._circle_polygon_contact
    OG._circle_polygon_contact = lambda *a: calls.append(1) or real(*a)
    try:
        _check_vs_oracle(case, ret, ga, gd)
    finally:
        OG._circle_polygon_contact = real
    assert len(calls) > 20  # circle x polygon resolutions in the compared gradients
