"""The scene parameter block (include/cotix_amd.h cotix_params) on CPU: the
reference's literals as defaults, the partitionable threefry layout pinned
by published JAX values, and every non-default parameter set
(tests/param_sets.py) bit-exact across the checkers -- the numpy oracle's
golden fixtures == the C port == the kernel's host emulation (every
envs-per-wave tiling) -- including the collider's contact choices.  The GPU
side is tests/test_gpu_params.py."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(HERE, "emu"))
sys.path.insert(0, GOLD)

from param_sets import PARAM_SETS, oracle_params  # noqa: E402

U = np.uint32
VARIANTS = ["_part", "_alt"]


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    import emu
    return emu, emu.load()


@pytest.fixture(scope="module")
def cp():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "..", "oracle")], check=True)
    from cotix_oracle import cport
    return cport, cport.load()


# ---------------------------------------------------------------------------
# the partitionable layout, pinned
# ---------------------------------------------------------------------------
def test_partitionable_published_values():
    """Published by the JAX documentation for the partitionable layout (the
    default from JAX 0.5; recalled here, not re-fetchable offline):
    split(key(0)) = [[1797259609, 2579123966], [928981903, 3453687069]],
    uniform(key(0)) = 0.947667, normal(key(42)) = -0.028304616.  The first
    row is also the Random123 KAT block threefry((0, 0), (0, 0))."""
    from cotix_oracle import params, prng
    with params.use(params.Params(prng_layout="partitionable")):
        assert prng.split(prng.PRNGKey(0)).tolist() == [[1797259609, 2579123966], [928981903, 3453687069]]
        assert prng.uniform(prng.PRNGKey(0), ()) == np.float32(0.947667)
        assert prng.normal(prng.PRNGKey(42), ())[()] == np.float32(-0.028304616)
        d = prng.gjk_initial_direction()
        assert [int(np.float32(v).view(U)) for v in d] == [0xBF607449, 0x3EF638CD]
    # and the legacy layout is untouched outside the block
    assert prng.split(prng.PRNGKey(0)).tolist() == [[4146024105, 967050713], [2718843009, 1272950319]]


def test_partitionable_split_at_and_bits():
    from cotix_oracle import params, prng
    with params.use(params.Params(prng_layout="partitionable")):
        for seed in (0, 3, 9):
            k = prng.PRNGKey(seed)
            for n in (1, 2, 5, 22):
                s = prng.split(k, n)
                for i in range(n):
                    assert (prng.split_at(k, n, i) == s[i]).all()
                    y0, y1 = prng.threefry2x32(k, np.array([0], U), np.array([i], U))
                    assert s[i].tolist() == [int(y0[0]), int(y1[0])]
            # random_bits of (m,) is the per-word block (0, i): a prefix of a longer draw
            assert (prng.random_bits(k, (7,))[:3] == prng.random_bits(k, (3,))).all()


def test_prng_part_fixture_regenerates():
    from cotix_oracle import params, prng
    g = np.load(os.path.join(GOLD, "prng_part.npz"))
    with params.use(params.Params(prng_layout="partitionable")):
        assert np.array_equal(np.array([prng.split(k, 5) for k in g["keys"][:16]], U), g["splits"])
        assert same_f32(np.array([prng.uniform(k, (7,), -3.0, 2.0) for k in g["keys"][:16]]), g["uniform7"])


# ---------------------------------------------------------------------------
# golden traces of the parameter sets: oracle fixture == C port == emulation
# ---------------------------------------------------------------------------
def _lunar_rows(make_scene, tr):
    from cotix_oracle import physics as P
    return np.ascontiguousarray(np.stack([make_scene(P.lunar_lander_bodies(k)) for k in tr["terrain_keys"]]))


@pytest.mark.parametrize("suffix", VARIANTS)
def test_variant_traces_regenerate(suffix):
    """The committed fixtures are the oracle's output under the block (a
    short prefix re-derived: 3 RoboCup envs x 4 steps)."""
    from cotix_oracle import params, prng
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "robocup_trace%s.npz" % suffix))
    with params.use(oracle_params(suffix)):
        d0 = prng.gjk_initial_direction()
        for e in range(3):
            bodies = P.robocup_bodies()
            for i, b in enumerate(bodies):
                b.set_dyn(tr["dyn"][0][e][i])
            key = tr["keys"][0][e]
            for t in range(4):
                trc = {}
                bodies, key = P.robocup_step(bodies, key, d0, G.ErrorFlag(), trc)
                assert same_f32([b.dyn() for b in bodies], tr["dyn"][t + 1][e]), (suffix, e, t)
                assert trc["chosen"] == list(tr["chosen"][t][e])


def _cport_trace(sc, tr, stages, geom=None):
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(U)
    err = np.zeros(dyn.shape[2], U)
    for t in range(tr["err"].shape[0]):
        ch, cl = sc.step_ex(dyn, keys, err, 1, stages, geom, trace=True, nthreads=2)
        assert np.array_equal(ch[0].T, tr["chosen"][t]), "chosen step %d" % t
        assert np.array_equal(cl[0].transpose(2, 0, 1), tr["cells"][t]), "cells step %d" % t
        assert same_f32(dyn.transpose(2, 0, 1), tr["dyn"][t + 1]), "step %d" % t
        assert np.array_equal(keys, tr["keys"][t + 1])
        assert np.array_equal(err, np.bitwise_or.reduce(tr["err"][: t + 1], axis=0))


@pytest.mark.parametrize("suffix", VARIANTS)
def test_cport_variant_traces(cp, suffix):
    cport, lib = cp
    from cotix_oracle import physics as P
    prm = oracle_params(suffix)
    _cport_trace(cport.Scene(lib, P.robocup_bodies(), prm), np.load(os.path.join(GOLD, "robocup_trace%s.npz" % suffix)),
                 cport.STAGES_ROBOCUP)
    tr = np.load(os.path.join(GOLD, "lunar_trace%s.npz" % suffix))
    rows = _lunar_rows(lambda b: cport.Scene(lib, b, prm).geom, tr)
    _cport_trace(cport.Scene(lib, P.lunar_lander_bodies(tr["terrain_keys"][0]), prm), tr, cport.STAGES_LUNAR, rows)


def _emu_trace(emu, lib, bodies, prm, geom_rows, tr, stages, EW):
    h, geom = emu.oracle_scene(lib, bodies, prm)
    gstride = 0
    if geom_rows is not None:
        geom, gstride = geom_rows, geom_rows.shape[1]
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(U)
    err = np.zeros(dyn.shape[2], U)
    for t in range(tr["err"].shape[0]):
        ch, cl = emu.step_ex(lib, h, dyn, keys, err, geom, gstride, 1, stages, len(bodies), E=EW)
        assert np.array_equal(ch[0].T, tr["chosen"][t]), "chosen step %d" % t
        assert np.array_equal(cl[0].transpose(2, 0, 1), tr["cells"][t]), "cells step %d" % t
        assert same_f32(dyn.transpose(2, 0, 1), tr["dyn"][t + 1]), "step %d" % t
        assert np.array_equal(keys, tr["keys"][t + 1]), "keys step %d" % t
        assert np.array_equal(err, np.bitwise_or.reduce(tr["err"][: t + 1], axis=0)), "err step %d" % t
    # the fused launch (key windows) == the per-step launches
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(U)
    err = np.zeros(dyn.shape[2], U)
    T = tr["err"].shape[0]
    ch, cl = emu.step_ex(lib, h, dyn, keys, err, geom, gstride, T, stages, len(bodies), E=EW)
    assert same_f32(dyn.transpose(2, 0, 1), tr["dyn"][T])
    assert np.array_equal(ch.transpose(0, 2, 1), tr["chosen"][:T])
    assert np.array_equal(cl.transpose(0, 3, 1, 2), tr["cells"][:T])


@pytest.mark.parametrize("EW", [1, 4, 8])
@pytest.mark.parametrize("suffix", VARIANTS)
def test_emu_variant_robocup(emu_lib, suffix, EW):
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    _emu_trace(emu, lib, P.robocup_bodies(), oracle_params(suffix), None,
               np.load(os.path.join(GOLD, "robocup_trace%s.npz" % suffix)), 1 | 4 | 16, EW)


@pytest.mark.parametrize("bp", [0, 32], ids=["full", "broadphase"])
@pytest.mark.parametrize("EW", [1, 4])
@pytest.mark.parametrize("suffix", VARIANTS)
def test_emu_variant_lunar(emu_lib, suffix, EW, bp):
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    prm = oracle_params(suffix)
    tr = np.load(os.path.join(GOLD, "lunar_trace%s.npz" % suffix))
    rows = _lunar_rows(lambda b: emu.oracle_scene(lib, b, prm)[1], tr).astype(np.float32)
    _emu_trace(emu, lib, P.lunar_lander_bodies(tr["terrain_keys"][0]), prm, rows, tr, 1 | 2 | 4 | 8 | 16 | bp, EW)


def test_default_block_is_the_legacy_trace(emu_lib):
    """An explicit block holding the reference's literals reproduces the
    default (legacy) golden trace: the defaults ARE the reference."""
    emu, lib = emu_lib
    from cotix_oracle import params
    from cotix_oracle import physics as P
    _emu_trace(emu, lib, P.robocup_bodies(), params.Params(), None,
               np.load(os.path.join(GOLD, "robocup_trace.npz")), 1 | 4 | 16, 4)


# ---------------------------------------------------------------------------
# GJK / EPA as operators (cotix/_collisions.py:277-329)
# ---------------------------------------------------------------------------
SUFFIXES = ["", "_part", "_alt"]


@pytest.mark.parametrize("suffix", SUFFIXES)
def test_gjk_epa_fixture_regenerates(suffix):
    from cotix_oracle import geometry as G
    from cotix_oracle import params, prng
    import make_golden as mg
    g = np.load(os.path.join(GOLD, "gjk_epa%s.npz" % suffix))
    pairs = mg.gjk_epa_pairs(np.random.default_rng(77))
    with params.use(oracle_params(suffix)):
        d0 = prng.gjk_initial_direction()
        for k in range(0, len(pairs), 7):
            a, b = pairs[k]
            h, s = G.check_for_collision_convex(a, b, d0)
            assert int(h) == g["hit"][k]
            assert same_f32(np.array(s, np.float32), g["simplex"][k])
            assert same_f32(G.epa(a, b, [tuple(v) for v in g["simplex"][k]], 11), g["pen11"][k])
    assert g["hit"].sum() > 250 and (1 - g["hit"]).sum() > 250


@pytest.mark.parametrize("suffix", SUFFIXES)
def test_cport_gjk_epa(cp, suffix):
    cport, lib = cp
    g = np.load(os.path.join(GOLD, "gjk_epa%s.npz" % suffix))
    a, b = np.ascontiguousarray(g["a"]), np.ascontiguousarray(g["b"])
    n = a.shape[0]
    hit = np.zeros(n, np.int32)
    sx = np.zeros((n, 3, 2), np.float32)
    prm = oracle_params(suffix).c_struct()
    lib.oracle_gjk(n, cport._p(a), cport._p(b), cport._p(hit), cport._p(sx), ctypes.cast(ctypes.pointer(prm), ctypes.c_void_p))
    assert np.array_equal(hit, g["hit"])
    assert same_f32(sx, g["simplex"])
    for it in (3, 11, 48):
        pen = np.zeros((n, 2), np.float32)
        s = np.ascontiguousarray(g["simplex"])
        assert lib.oracle_epa(n, cport._p(a), cport._p(b), cport._p(s), it, cport._p(pen)) == 0
        assert same_f32(pen, g["pen%d" % it]), it


@pytest.mark.parametrize("suffix", SUFFIXES)
def test_emu_gjk_epa(emu_lib, suffix):
    """The device code of cotix_gjk / cotix_epa (host build) vs the fixtures."""
    emu, lib = emu_lib
    g = np.load(os.path.join(GOLD, "gjk_epa%s.npz" % suffix))
    a, b = np.ascontiguousarray(g["a"]), np.ascontiguousarray(g["b"])
    n = a.shape[0]
    hit = np.zeros(n, np.int32)
    sx = np.zeros((n, 3, 2), np.float32)
    lib.emu_gjk(n, emu._p(a), emu._p(b), emu._p(hit), emu._p(sx), emu.params_ref(oracle_params(suffix)))
    assert np.array_equal(hit, g["hit"])
    assert same_f32(sx, g["simplex"])
    for it in (3, 11, 48):
        pen = np.zeros((n, 2), np.float32)
        s = np.ascontiguousarray(g["simplex"])
        assert lib.emu_epa(n, emu._p(a), emu._p(b), emu._p(s), it, emu._p(pen)) == 0
        assert same_f32(pen, g["pen%d" % it]), it
    assert lib.emu_epa(n, emu._p(a), emu._p(b), emu._p(s), 2, emu._p(pen)) != 0  # error_if: fewer than 3


@pytest.mark.parametrize("name", ["poly_poly", "aabb_poly", "circle_poly"])
def test_contacts_alt_params_emu_vs_cport(emu_lib, cp, name):
    """The polygon contact operators under the non-default block (GJK capped
    at 1 step, EPA at 3 iterations; circle x polygon EPA 128 -> 20): the
    device code == the C port, and the block changes results."""
    emu, elib = emu_lib
    cport, clib = cp
    from cotix_oracle import params
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a, b = np.ascontiguousarray(g[name + "_a"]), np.ascontiguousarray(g[name + "_b"])
    n, fn = a.shape[0], int(g[name + "_fn"])
    prm = params.Params(**dict(PARAM_SETS["_alt"], epa_circle_iters=20))
    outs = []
    for lib, f, ref in ((elib, elib.emu_contacts_ex, emu.params_ref), (clib, clib.oracle_contacts_ex,
                                                                      cport.params_ref)):
        out = np.zeros((n, 4), np.float32)
        err = np.zeros(n, np.uint32)
        f(fn, n, emu._p(a), emu._p(b), emu._p(out), emu._p(err), ref(prm))
        outs.append(out)
    assert same_f32(outs[0], outs[1])
    assert not same_f32(outs[0], g[name + "_out"])


# ---------------------------------------------------------------------------
# the C-ABI's parameter block
# ---------------------------------------------------------------------------
def test_capi_params_defaults_and_checks():
    import parallax_amd as pa
    lib = pa._ffi.lib
    c = pa.params.CotixParams()
    assert lib.cotix_params_default(ctypes.byref(c)) == 0
    assert pa.Params.from_c(c) == pa.Params()  # the reference's literals
    assert (c.baumgarte, c.baumgarte_dt, c.contact_p) == (np.float32(0.3), np.float32(0.01), 0.5)
    assert (c.prng_layout, c.gjk_max_steps, c.epa_max_iters, c.epa_circle_iters, c.epa_body_iters) == (0, 32, 48,
                                                                                                       128, 48)
    bodies = pa.scenarios.robocup_bodies()
    for sfx in ("", "_part", "_alt"):
        p = pa.Params(**PARAM_SETS[sfx])
        assert pa.Scene(bodies, p).compiled_params() == p
    for bad in ({"gjk_max_steps": -1}, {"epa_max_iters": 2}, {"epa_circle_iters": 129}, {"epa_body_iters": 0}):
        with pytest.raises(RuntimeError, match="outside"):
            pa.Scene(bodies, pa.Params(**bad))
    with pytest.raises(ValueError):
        pa.Params(prng_layout="threefry")
    c.prng_layout = 7  # the block is checked before anything else
    h = ctypes.c_void_p()
    assert lib.cotix_scene_create_ex(1, None, 0, None, None, None, ctypes.byref(c), ctypes.byref(h)) != 0
    assert b"prng_layout" in lib.cotix_last_error()


@pytest.mark.parametrize("suffix", ["", "_part"])
def test_gjk_start_direction_fixture_oracle_and_device_code(suffix):
    """check_for_collision_convex(a, b, initial_direction, key)
    (cotix/_collisions.py:277-298): the fixture's start directions equal the
    oracle's gjk_start_direction and the kernel's device code (cx::
    random_direction / cx::gjk_start, host build) bit for bit; key
    PRNGKey(1) gives the default constant; a sample of the hit / simplex
    rows re-derives from the oracle."""
    import emu
    from cotix_oracle import geometry as G
    from cotix_oracle import params as PR
    from cotix_oracle import prng
    import make_golden as M
    g = np.load(os.path.join(GOLD, "gjk_dir%s.npz" % suffix))
    n = len(g["hit"])
    p = oracle_params(suffix) if suffix else None
    with PR.use(p):
        want = np.array([prng.gjk_start_direction(g["init"][i], g["keys"][i]) for i in range(n)], np.float32)
        assert same_f32(want, g["start"])
        assert tuple(prng.random_direction(prng.PRNGKey(1))) == tuple(prng.gjk_initial_direction())
        pairs = M.gjk_epa_pairs(np.random.default_rng(91))[::2]
        for i in range(0, n, 37):
            h, sx = G.check_for_collision_convex(pairs[i][0], pairs[i][1], tuple(g["start"][i]))
            assert int(h) == int(g["hit"][i]) and same_f32(np.array(sx, np.float32).reshape(3, 2), g["simplex"][i]), i
    lib = emu.load()
    P = ctypes.c_void_p
    keys = np.ascontiguousarray(g["keys"], np.uint32)
    init = np.ascontiguousarray(g["init"], np.float32)
    out = np.zeros((n, 2), np.float32)
    lib.emu_gjk_start(n, keys.ctypes.data_as(P), init.ctypes.data_as(P), 1 if suffix else 0, out.ctypes.data_as(P))
    assert same_f32(out, g["start"])


def test_erf_inv_cr_reproduces_published_normals():
    """random_direction's erf_inv (correctly rounded log1p) gives the same 13
    published jax.random.normal(PRNGKey(0), .) values as erf_inv32."""
    from cotix_oracle import prng
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    for shape, exp in (((10,), [-0.3721109, 0.26423115, -0.18252768, -0.7368197, -0.44030377, -0.1521442,
                                -0.67135346, -0.5908641, 0.73168886, 0.5673026]),
                       ((3,), [1.8160863, -0.48262316, 0.33988908])):
        u = prng.uniform(prng.PRNGKey(0), shape, lo, 1.0)
        got = [np.float32(np.float32(np.sqrt(2.0)) * prng.erf_inv32_cr(v)) for v in u]
        assert got == np.array(exp, np.float32).tolist()
