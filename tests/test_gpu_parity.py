"""GPU parity of the HIP hot path (through the C-ABI) against the oracle.

Bar (DESIGN.md "Parity"): float32 results bit-identical to the oracle --
equal bit patterns, and NaN exactly where the oracle has NaN (NaN payloads
are not compared) -- plus identical error bits, keys and contact choices:
the collider trace of cotix_step_ex (the chosen partner j* of every body at
every step, cotix/_colliders.py:274-295, and the winning scan candidate of
every all_contacts cell, :208-268) is compared with the golden traces and
the C port wherever a trajectory is.  This is stricter than north_star's
1e-5 relative tolerance.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def same_f32(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def diff_report(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    bad = ~((np.isnan(a) & np.isnan(b)) | (a.view(np.uint32) == b.view(np.uint32)))
    idx = np.argwhere(bad)[:5]
    return "first mismatches: " + "; ".join("%s: %r vs %r" % (tuple(i), a[tuple(i)], b[tuple(i)]) for i in idx)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a visible GPU (torch.cuda.is_available() is False)")
    return torch


def u32_to_i32(x):
    return np.asarray(x, np.uint32).view(np.int32)


# ---------------------------------------------------------------------------
# operators
# ---------------------------------------------------------------------------
def test_prng_kernels(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "prng.npz"))
    keys = torch.tensor(u32_to_i32(g["keys"]), device="cuda")
    ctr = torch.tensor(u32_to_i32(g["ctr"]), device="cuda")
    out = pa.random.threefry2x32(keys, ctr).cpu().numpy().view(np.uint32)
    assert np.array_equal(out, g["blocks"])
    sp = pa.random.split(keys[:16], 5).cpu().numpy().view(np.uint32)
    assert np.array_equal(sp, g["splits"])
    assert same_f32(pa.random.uniform(keys[:16], 7, -3.0, 2.0).cpu().numpy(), g["uniform7"])
    assert same_f32(pa.random.uniform(keys[:16], None, 4.0, 8.0).cpu().numpy(), g["uniform1"])
    # published: split(PRNGKey(0)) and uniform(PRNGKey(0), (3,))
    k0 = pa.random.PRNGKey(0, "cuda")
    assert pa.random.split(k0).cpu().numpy().view(np.uint32).tolist() == [[4146024105, 967050713],
                                                                          [2718843009, 1272950319]]
    assert same_f32(pa.random.uniform(k0, 3).cpu().numpy(), np.array([0.9653214, 0.31468165, 0.63302994], np.float32))


@pytest.mark.parametrize("name", ["aabb_aabb", "circle_circle", "circle_aabb", "poly_poly", "aabb_poly",
                                  "circle_poly"])
def test_contact_operators(torch_cuda, name):
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a = torch.tensor(g[name + "_a"], device="cuda")
    b = torch.tensor(g[name + "_b"], device="cuda")
    info, err = pa.run_contacts(int(g[name + "_fn"]), a, b)
    got = torch.cat([info.penetration_vector, info.contact_point], 1).cpu().numpy()
    assert same_f32(got, g[name + "_out"]), diff_report(got, g[name + "_out"])
    assert np.array_equal(err.cpu().numpy(), g[name + "_err"])


def test_resolve_operator(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    rng = np.random.default_rng(3)
    n = 400
    d1 = rng.normal(size=(n, 6)).astype(np.float32)
    d2 = rng.normal(size=(n, 6)).astype(np.float32)
    p1 = np.abs(rng.normal(size=(n, 4))).astype(np.float32) + 0.1
    p2 = np.abs(rng.normal(size=(n, 4))).astype(np.float32) + 0.1
    p2[::7, 0] = np.inf  # static partner (mass inf) as in both scenarios
    c = rng.normal(size=(n, 4)).astype(np.float32)
    c[::11, 2] = np.nan  # no-contact rows are a no-op
    want1, want2 = d1.copy(), d2.copy()
    for k in range(n):
        b1 = P.Body([], *p1[k, :2], elasticity=p1[k, 2], friction_coefficient=p1[k, 3])
        b2 = P.Body([], *p2[k, :2], elasticity=p2[k, 2], friction_coefficient=p2[k, 3])
        b1.set_dyn(d1[k])
        b2.set_dyn(d2[k])
        P.resolve_collision(b1, b2, ((c[k, 0], c[k, 1]), (c[k, 2], c[k, 3])))
        want1[k], want2[k] = b1.dyn(), b2.dyn()
    t1, t2 = torch.tensor(d1, device="cuda"), torch.tensor(d2, device="cuda")
    pa.resolve_collision(t1, torch.tensor(p1, device="cuda"), t2, torch.tensor(p2, device="cuda"),
                         torch.tensor(c, device="cuda"))
    assert same_f32(t1.cpu().numpy(), want1), diff_report(t1.cpu().numpy(), want1)
    assert same_f32(t2.cpu().numpy(), want2), diff_report(t2.cpu().numpy(), want2)


def test_order_clockwise_operator(torch_cuda):
    torch = torch_cuda
    from cotix_oracle import geometry as G
    import parallax_amd as pa
    rng = np.random.default_rng(8)
    for nv in (3, 4, 6, 8):
        xy = rng.normal(size=(300, nv, 2)).astype(np.float32)
        t = torch.tensor(xy, device="cuda")
        pa._ffi.check(pa._ffi.lib.cotix_order_clockwise(pa._ffi.ptr(t), 300, nv, pa._ffi.stream_ptr()), "ocw")
        want = np.array([G.order_clockwise([tuple(v) for v in p]) for p in xy], np.float32)
        assert same_f32(t.cpu().numpy(), want)


# ---------------------------------------------------------------------------
# multi-step traces (fused kernel) vs the golden oracle traces
# ---------------------------------------------------------------------------
def _check_trace(world, tr, stages, T, per_step=True):
    """State, keys, error bits AND the collider's choices (j* per body, winning
    candidate per cell) of every step against the golden oracle trace."""
    import torch
    if per_step:
        for t in range(T):
            trc = {}
            world.step(1, 1e-2, stages, trace=trc)
            torch.cuda.synchronize()
            dyn = world.dyn.permute(2, 0, 1).cpu().numpy()
            assert same_f32(dyn, tr["dyn"][t + 1]), "step %d: %s" % (t, diff_report(dyn, tr["dyn"][t + 1]))
            keys = world.keys.cpu().numpy().view(np.uint32)
            assert np.array_equal(keys, tr["keys"][t + 1]), "step %d keys" % t
            err = world.err.cpu().numpy()
            want_err = np.bitwise_or.reduce(tr["err"][: t + 1], axis=0)
            assert np.array_equal(err, want_err), "step %d err %s vs %s" % (t, err, want_err)
            assert np.array_equal(trc["chosen"][0].T.cpu().numpy(), tr["chosen"][t]), "step %d chosen" % t
            assert np.array_equal(trc["cells"][0].permute(2, 0, 1).cpu().numpy(), tr["cells"][t]), "step %d cells" % t
    else:
        trc = {}
        world.step(T, 1e-2, stages, trace=trc)
        torch.cuda.synchronize()
        dyn = world.dyn.permute(2, 0, 1).cpu().numpy()
        assert same_f32(dyn, tr["dyn"][T]), diff_report(dyn, tr["dyn"][T])
        assert np.array_equal(world.keys.cpu().numpy().view(np.uint32), tr["keys"][T])
        assert np.array_equal(trc["chosen"].permute(0, 2, 1).cpu().numpy(), tr["chosen"][:T]), "fused chosen"
        assert np.array_equal(trc["cells"].permute(0, 3, 1, 2).cpu().numpy(), tr["cells"][:T]), "fused cells"


@pytest.mark.parametrize("per_step", [True, False])
def test_robocup_trace(torch_cuda, per_step):
    torch = torch_cuda
    import parallax_amd as pa
    tr = np.load(os.path.join(GOLD, "robocup_trace.npz"))
    T, B = tr["err"].shape
    env = pa.RoboCupEnv(batch=B, device="cuda", keys=torch.tensor(u32_to_i32(tr["keys"][0]), device="cuda"),
                        perturb=True)
    assert same_f32(env.world.dyn.permute(2, 0, 1).cpu().numpy(), tr["dyn"][0]), "perturbed reset state"
    _check_trace(env.world, tr, env.stages, T, per_step)


@pytest.mark.parametrize("per_step", [True, False])
def test_lunar_trace(torch_cuda, per_step):
    torch = torch_cuda
    import parallax_amd as pa
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    T, B = tr["err"].shape
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tr["terrain_keys"]), device="cuda"), batch=B, device="cuda",
                        collider_keys=torch.tensor(u32_to_i32(tr["keys"][0]), device="cuda"))
    ll.world.dyn.copy_(torch.tensor(tr["init"], device="cuda").permute(1, 2, 0))
    _check_trace(ll.world, tr, ll.stages, T, per_step)


def test_lunar_terrain_matches_oracle(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    keys = prng.split(prng.PRNGKey(0), 16)
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(keys), device="cuda"), batch=16, device="cuda")
    geom = ll.world.geom.cpu().numpy()
    for e in range(16):
        ref = P.lunar_lander_bodies(keys[e])
        want = np.concatenate([np.array(p.vertices_, np.float32).ravel() for b in ref for p in b.parts])
        assert same_f32(geom[e], want), "env %d: %s" % (e, diff_report(geom[e], want))


def test_box_world_trace(torch_cuda):
    """Generic scene with finite dynamics (balls in a box)."""
    torch = torch_cuda
    import parallax_amd as pa
    sys_path = os.path.join(GOLD)
    import sys
    sys.path.insert(0, sys_path)
    import make_golden as mg
    tr = np.load(os.path.join(GOLD, "box_world_trace.npz"))
    T, B = tr["err"].shape
    for e in range(B):
        ob = mg.box_world_bodies(e)
        bodies = []
        for b in ob:
            parts = []
            for p in b.parts:
                if p.kind == "AABB":
                    parts.append(pa.AABB(list(p.lower), list(p.upper)))
                else:
                    parts.append(pa.Circle(p.radius, list(p.position)))
            bodies.append(pa.AnyBody(shape=pa.UniversalShape(*parts), mass=b.mass, inertia=b.inertia,
                                     position=list(b.position), velocity=list(b.velocity), angle=b.angle,
                                     angular_velocity=b.angular_velocity, elasticity=b.elasticity,
                                     friction_coefficient=b.friction_coefficient))
        w = pa.World(bodies, 1, "cuda", torch.tensor(u32_to_i32(tr["keys"][0][e:e + 1]), device="cuda"))
        sub = {k: tr[k][:, e:e + 1] for k in ("dyn", "keys", "err", "chosen", "cells")}
        _check_trace(w, sub, pa._ffi.STAGES_ROBOCUP, T, per_step=True)


# ---------------------------------------------------------------------------
# operator composition == fused kernel (the reference's call sequence)
# ---------------------------------------------------------------------------
def test_operator_composition_matches_fused(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    B = tr["err"].shape[1]
    mk = lambda: pa.LunarLander(key=torch.tensor(u32_to_i32(tr["terrain_keys"]), device="cuda"),  # noqa: E731
                                batch=B, device="cuda",
                                collider_keys=torch.tensor(u32_to_i32(tr["keys"][0]), device="cuda"))
    fused, ops = mk(), mk()
    for x in (fused, ops):
        x.world.dyn.copy_(torch.tensor(tr["init"], device="cuda").permute(1, 2, 0))
    physics, collider = pa.ExplicitEulerPhysics(), pa.RandomizedCollider()
    for t in range(6):
        fused.world.step(1, 1e-2, fused.stages)
        # examples/test_viz.py:24-44 composed from the operators
        w, _ = physics.step(ops.world, dt=1e-2)
        w.dyn[0, 3] += -0.002
        w.dyn[0, 2] += 0.0
        collider.resolve(w, w.keys)
        w.keys.copy_(pa.random.split(w.keys)[:, 0])
        ops.step()
    torch.cuda.synchronize()
    assert same_f32(ops.world.dyn.cpu().numpy(), fused.world.dyn.cpu().numpy())
    assert torch.equal(ops.world.keys, fused.world.keys)


# ---------------------------------------------------------------------------
# BASELINE sizes: 4096 envs -- sampled oracle parity + size-independent properties
# ---------------------------------------------------------------------------
def _oracle_envs(make_bodies, step_fn, init_dyn, keys, env_ids, T):
    from cotix_oracle import geometry as G
    from cotix_oracle import prng
    d0 = prng.gjk_initial_direction()
    out = []
    for e in env_ids:
        b = make_bodies(e)
        for i in range(len(b)):
            b[i].set_dyn(init_dyn[e][i])
        k = np.array(keys[e], np.uint32)
        err = G.ErrorFlag()
        for _ in range(T):
            b, k = step_fn(b, k, d0, err)
        out.append((np.array([x.dyn() for x in b], np.float32), k, err.bits))
    return out


def test_robocup_4096_sampled_oracle_and_properties(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    B, T = 4096, 6
    env = pa.RoboCupEnv(batch=B, device="cuda", perturb=True)
    init = env.world.dyn.permute(2, 0, 1).cpu().numpy().copy()
    keys0 = env.world.keys.cpu().numpy().view(np.uint32).copy()
    env.world.step(T, 1e-2, env.stages)
    torch.cuda.synchronize()
    dyn = env.world.dyn.permute(2, 0, 1).cpu().numpy()
    err = env.world.err.cpu().numpy()
    ids = [0, 1, 2, 777, 2048, 4095]
    for e, (d, k, eb) in zip(ids, _oracle_envs(lambda e: P.robocup_bodies(), P.robocup_step, init, keys0, ids, T)):
        assert same_f32(dyn[e], d), "env %d: %s" % (e, diff_report(dyn[e], d))
        assert np.array_equal(env.world.keys[e].cpu().numpy().view(np.uint32), k)
        assert err[e] == eb
    # determinism + placement independence: the same envs, reversed order, in a fresh world
    env2 = pa.RoboCupEnv(batch=B, device="cuda", keys=env.world.keys.new_tensor(keys0.view(np.int32)).flip(0))
    env2.world.dyn.copy_(torch.tensor(init, device="cuda").flip(0).permute(1, 2, 0))
    env2.world.step(T, 1e-2, env2.stages)
    assert same_f32(env2.world.dyn.permute(2, 0, 1).flip(0).cpu().numpy(), dyn)
    # fused T steps == T single-step launches
    env3 = pa.RoboCupEnv(batch=B, device="cuda", perturb=True)
    for _ in range(T):
        env3.world.step(1, 1e-2, env3.stages)
    assert same_f32(env3.world.dyn.cpu().numpy(), env.world.dyn.cpu().numpy())


def test_lunar_4096_sampled_oracle(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    B, T = 4096, 4
    tkeys = prng.split(prng.PRNGKey(0), B)
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tkeys), device="cuda"), batch=B, device="cuda")
    # drop a quarter of the landers onto the ground so GJK/EPA contacts fire
    drop = torch.zeros(B, device="cuda")
    drop[::4] = 6.3
    for i in range(3):
        ll.world.dyn[i, 1] -= drop
        ll.world.dyn[i, 3] = torch.where(drop > 0, torch.tensor(-0.3, device="cuda"), ll.world.dyn[i, 3])
    init = ll.world.dyn.permute(2, 0, 1).cpu().numpy().copy()
    keys0 = ll.world.keys.cpu().numpy().view(np.uint32).copy()
    ll.world.step(T, 1e-2, ll.stages)
    torch.cuda.synchronize()
    dyn = ll.world.dyn.permute(2, 0, 1).cpu().numpy()
    ids = [0, 4, 8, 1001, 2052, 4092, 4095]
    res = _oracle_envs(lambda e: P.lunar_lander_bodies(tkeys[e]), P.lunar_lander_step, init, keys0, ids, T)
    for e, (d, k, eb) in zip(ids, res):
        assert same_f32(dyn[e], d), "env %d: %s" % (e, diff_report(dyn[e], d))


# ---------------------------------------------------------------------------
# BASELINE sizes, every env: HIP path vs the C port of the oracle
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cport_lib():
    """The C port of the oracle.  A missing build is a FAILURE under -m gpu,
    never a skip: these tests are the north star's index-parity evidence."""
    from cotix_oracle import cport
    assert os.path.exists(cport.LIB), ("oracle C port %s missing: build it before the GPU run "
                                       "(python __graft_entry__.py, or make -C oracle)" % cport.LIB)
    return cport, cport.load()


def _robocup_vs_cport(torch, pa, cport, lib, env, dyn, keys, launches, T, actions=None):
    """Steps a BatchedEnv (autoreset) and the C port side by side; compares
    state, keys, err, restart counts and the collider trace of every launch."""
    from cotix_oracle import physics as P
    B = dyn.shape[2]
    reset = dyn.copy()
    err = np.zeros(B, np.uint32)
    resets = np.zeros(B, np.uint32)
    sc = cport.Scene(lib, P.robocup_bodies())
    for q in range(launches):
        act = None if actions is None else actions[q]
        trc = {}
        env.step(T, action=None if act is None else torch.tensor(act, device="cuda"), trace=trc)
        wch, wcl = sc.step_ex(dyn, keys, err, T, cport.STAGES_ROBOCUP, None, act, 4, reset, resets, trace=True,
                              nthreads=16)
        torch.cuda.synchronize()
        assert np.array_equal(trc["chosen"].cpu().numpy(), wch), "launch %d chosen" % q
        assert np.array_equal(trc["cells"].cpu().numpy(), wcl), "launch %d cells" % q
    got = env.world.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(env.world.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(env.world.err.cpu().numpy().view(np.uint32), err)
    assert np.array_equal(env.resets.cpu().numpy().view(np.uint32), resets)
    assert resets.sum() > 0
    return wch, wcl


def test_robocup_4096_all_envs_vs_cport_autoreset(torch_cuda, cport_lib):
    """The bench workload itself: 4096 perturbed envs, 3 launches x 16 fused
    steps with episode restarts, compared for every env -- state, keys, error
    bits, restarts and every contact choice (j* per body, winner per cell)."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    B = 4096
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True), autoreset=True)
    env.reset()
    dyn = np.ascontiguousarray(env.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(env.world.keys.cpu().numpy().view(np.uint32))
    ch, cl = _robocup_vs_cport(torch, pa, cport, lib, env, dyn, keys, 3, 16)
    assert (ch != np.arange(5)[None, :, None]).any() and (cl >= 0).any()


def test_robocup_actions_with_autoreset_vs_cport(torch_cuda, cport_lib):
    """An RL loop: BatchedEnv.step(action) with autoreset (ball dv actions
    N(0, 0.1^2)), 4096 envs, 2 launches x 12 steps, vs the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    B, T = 4096, 12
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True), autoreset=True)
    env.reset()
    dyn = np.ascontiguousarray(env.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(env.world.keys.cpu().numpy().view(np.uint32))
    rng = np.random.default_rng(12)
    acts = [np.ascontiguousarray((rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)) for _ in range(2)]
    _robocup_vs_cport(torch, pa, cport, lib, env, dyn, keys, 2, T, acts)


def test_config4_shard_8192_vs_cport(torch_cuda, cport_lib):
    """BASELINE config 4 on one GPU: the per-GPU shard of the 65,536-env run
    (B = 8192, global ids 3*8192 .. 4*8192-1, built from those ids as bench.py
    --gpus 8 builds rank 3) with restarts, every env vs the C port fed the
    same global ids; 2 launches x 16 steps."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    B, rank, world = 8192, 3, 8
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True, env_offset=rank * B,
                                      total_envs=world * B), autoreset=True)
    env.reset()
    dyn, keys = cport.robocup_batch(B, offset=rank * B, total=world * B)
    assert same_f32(env.world.dyn.cpu().numpy(), dyn), "shard reset state"
    assert np.array_equal(env.world.keys.cpu().numpy().view(np.uint32), keys), "shard keys"
    _robocup_vs_cport(torch, pa, cport, lib, env, np.ascontiguousarray(dyn), np.ascontiguousarray(keys), 2, 16)


def test_lunar_4096_all_envs_vs_cport(torch_cuda, cport_lib):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    cport, lib = cport_lib
    B, T = 4096, 8
    tkeys = prng.split(prng.PRNGKey(0), B)
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tkeys), device="cuda"), batch=B, device="cuda")
    drop = torch.zeros(B, device="cuda")
    drop[::3] = 6.25
    for i in range(3):
        ll.world.dyn[i, 1] -= drop
        ll.world.dyn[i, 3] = torch.where(drop > 0, torch.tensor(-0.3, device="cuda"), ll.world.dyn[i, 3])
    dyn = np.ascontiguousarray(ll.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(ll.world.keys.cpu().numpy().view(np.uint32))
    geom = np.ascontiguousarray(ll.world.geom.cpu().numpy())
    err = np.zeros(B, np.uint32)
    trc = {}
    ll.world.step(T, 1e-2, ll.stages, trace=trc)
    sc = cport.Scene(lib, P.lunar_lander_bodies(tkeys[0]))
    wch, wcl = sc.step_ex(dyn, keys, err, T, cport.STAGES_LUNAR, geom, trace=True, nthreads=16)
    torch.cuda.synchronize()
    got = ll.world.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(ll.world.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(ll.world.err.cpu().numpy().view(np.uint32), err)
    assert (wcl >= 0).sum() > B
    assert np.array_equal(trc["chosen"].cpu().numpy(), wch)
    assert np.array_equal(trc["cells"].cpu().numpy(), wcl)


def test_lunar_restarts_move_static_body_vs_cport(torch_cuda, cport_lib):
    """Phase T keeps a body's world parts while its pose bits are unchanged
    (LunarLander's static terrain).  4096 envs dropped onto the terrain, 2
    launches x 9 steps with restarts into a reset state whose terrain body is
    shifted (even envs) or only rotated (odd envs), and a NaN-posed lander in
    some: every env, restart count and contact choice vs the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    cport, lib = cport_lib
    B, T = 4096, 9
    tkeys = prng.split(prng.PRNGKey(4), B)
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tkeys), device="cuda"), batch=B, device="cuda")
    w = ll.world
    for i in range(3):
        w.dyn[i, 1] -= 6.3
        w.dyn[i, 3] = -0.3
    reset = w.dyn.clone()
    reset[3, 0, 0::2] += 0.75
    reset[3, 4, 1::2] = 2.0
    reset[0, 4, 3::5] = float("nan")
    w.err[1::3] = 1
    dyn = np.ascontiguousarray(w.dyn.cpu().numpy())
    keys = np.ascontiguousarray(w.keys.cpu().numpy().view(np.uint32))
    err = np.ascontiguousarray(w.err.cpu().numpy().view(np.uint32))
    geom = np.ascontiguousarray(w.geom.cpu().numpy())
    rst = np.ascontiguousarray(reset.cpu().numpy())
    resets = torch.zeros(B, dtype=torch.int32, device="cuda")
    want_resets = np.zeros(B, np.uint32)
    sc = cport.Scene(lib, P.lunar_lander_bodies(tkeys[0]))
    for q in range(2):
        trc = {}
        w.step(T, 1e-2, ll.stages, dyn_reset=reset, resets=resets, trace=trc)
        wch, wcl = sc.step_ex(dyn, keys, err, T, cport.STAGES_LUNAR, geom, None, 0, rst, want_resets, trace=True,
                              nthreads=16)
        torch.cuda.synchronize()
        assert np.array_equal(trc["chosen"].cpu().numpy(), wch), "launch %d chosen" % q
        assert np.array_equal(trc["cells"].cpu().numpy(), wcl), "launch %d cells" % q
        if q == 0:
            w.err[0::4] = 1
            err[0::4] = 1
    got = w.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(w.err.cpu().numpy().view(np.uint32), err)
    assert np.array_equal(resets.cpu().numpy().view(np.uint32), want_resets)
    assert want_resets.sum() == len(range(1, B, 3)) + len(range(0, B, 4))


def test_config1_lunar_single_env_10000_steps_vs_cport(torch_cuda, cport_lib):
    """BASELINE config 1 (examples/test_viz.py:24-48): one LunarLander env,
    terrain PRNGKey(0), collider key chain from PRNGKey(0), dt 1e-2, gravity
    0.002, 10,000 driver steps -- the GPU (20 launches x 500 fused steps) vs
    the C port bit for bit: the state after every launch and the collider's
    choices at every one of the 10,000 steps."""
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    cport, lib = cport_lib
    ll = pa.LunarLander(batch=1, device="cuda")  # key PRNGKey(0); collider key PRNGKey(0)
    sc = cport.Scene(lib, P.lunar_lander_bodies(prng.PRNGKey(0)))
    dyn = np.ascontiguousarray(ll.world.dyn.cpu().numpy())
    want0 = np.array([b.dyn() for b in P.lunar_lander_bodies(prng.PRNGKey(0))], np.float32)[:, :, None]
    assert same_f32(dyn, want0)
    keys = np.ascontiguousarray(ll.world.keys.cpu().numpy().view(np.uint32))
    assert keys.tolist() == [[0, 0]]
    geom = np.ascontiguousarray(ll.world.geom.cpu().numpy()[None] if ll.world.geom.dim() == 1
                                else ll.world.geom.cpu().numpy())
    err = np.zeros(1, np.uint32)
    contacts = 0
    for q in range(20):
        trc = {}
        ll.world.step(500, 1e-2, ll.stages, trace=trc)
        wch, wcl = sc.step_ex(dyn, keys, err, 500, cport.STAGES_LUNAR, geom, trace=True, nthreads=1)
        torch.cuda.synchronize()
        got = ll.world.dyn.cpu().numpy()
        assert same_f32(got, dyn), "after step %d: %s" % (500 * (q + 1), diff_report(got, dyn))
        assert np.array_equal(ll.world.keys.cpu().numpy().view(np.uint32), keys)
        assert np.array_equal(ll.world.err.cpu().numpy().view(np.uint32), err)
        assert np.array_equal(trc["chosen"].cpu().numpy(), wch), "chosen, launch %d" % q
        assert np.array_equal(trc["cells"].cpu().numpy(), wcl), "cells, launch %d" % q
        contacts += int((wcl >= 0).sum())
    assert contacts > 0  # the lander reached the terrain (GJK/EPA contacts)


# ---------------------------------------------------------------------------
# differentiable rollout (BASELINE config 5)
# ---------------------------------------------------------------------------
def _gpu_rollout(torch, case, bodies_pa, want_dyn0=True, stages=None, world=None, envs_per_wave=0):
    import parallax_amd as pa
    B = case["S0"].shape[0]
    keys = torch.tensor(u32_to_i32(case["keys"]), device="cuda")
    w = pa.World(bodies_pa, B, "cuda", keys) if world is None else world
    if envs_per_wave:
        w.set_variant(envs_per_wave)
    if world is not None:
        w.keys.copy_(keys)
    w.dyn.copy_(torch.tensor(case["S0"], device="cuda").permute(1, 2, 0))
    acts = torch.tensor(case["actions"], device="cuda")
    ret, saved = pa.rollout_forward(w, acts, case["ab"], case["w"],
                                    stages=pa._ffi.STAGES_ROBOCUP if stages is None else stages)
    ga, gd = pa.rollout_backward(w, saved, want_dyn0=want_dyn0)
    _check_tape_vs_replay(pa, w, saved, ga, gd)
    return w, ret.cpu().numpy(), ga.cpu().numpy(), (gd.cpu().numpy() if gd is not None else None), saved


def _check_tape_vs_replay(pa, world, saved, ga, gd):
    """The backward from the forward's tape (what the library runs) equals the
    re-play of the forward (MODE 2) bit for bit, NaN patterns included."""
    import torch
    assert saved["tape"] is not None
    ra, rd = pa.rollout_backward(world, saved, want_dyn0=gd is not None, replay=True)
    torch.cuda.synchronize()
    assert same_f32(ga.cpu().numpy(), ra.cpu().numpy()), diff_report(ga.cpu().numpy(), ra.cpu().numpy())
    if gd is not None:
        assert same_f32(gd.cpu().numpy(), rd.cpu().numpy()), diff_report(gd.cpu().numpy(), rd.cpu().numpy())


def _pa_part(pa, p):
    if p.kind == "AABB":
        return pa.AABB(list(p.lower), list(p.upper))
    if p.kind == "Circle":
        return pa.Circle(p.radius, list(p.position))
    return getattr(pa, p.kind)([list(v) for v in p.vertices_], presorted=True)


def _pa_bodies(pa, oracle_bodies):
    out = []
    for b in oracle_bodies:
        parts = [_pa_part(pa, p) for p in b.parts]
        out.append(pa.AnyBody(shape=pa.UniversalShape(*parts), mass=b.mass, inertia=b.inertia,
                              position=list(b.position), velocity=list(b.velocity), angle=b.angle,
                              angular_velocity=b.angular_velocity, elasticity=b.elasticity,
                              friction_coefficient=b.friction_coefficient))
    return out


def test_rollout_grad_box_world_vs_oracle(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.box_case(6, 32, seed=1)
    _, ret, ga, gd, _ = _gpu_rollout(torch, case, _pa_bodies(pa, case["make"]()))
    orc = GC.oracle(case)
    for e in orc:
        r, oga, ogS = orc[e]
        assert np.float32(ret[e]).view(np.uint32) == np.float32(r).view(np.uint32), (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d grad_action %s" % (e, msg)
        ok, msg = GC.close(gd[:, :, e], ogS, case["tol"], case["name"])
        assert ok, "env %d grad_dyn0 %s" % (e, msg)


def _check_grad_vs_oracle(case, ret, ga, gd):
    import grad_cases as GC
    orc = GC.oracle(case)
    for e in orc:
        r, oga, ogS = orc[e]
        assert np.float32(ret[e]).view(np.uint32) == np.float32(r).view(np.uint32), (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d grad_action %s" % (e, msg)
        ok, msg = GC.close(gd[:, :, e], ogS, case["tol"], case["name"])
        assert ok, "env %d grad_dyn0 %s" % (e, msg)


def test_rollout_grad_lunar_vs_oracle(torch_cuda):
    """Gradients through GJK/EPA polygon contacts and the LunarLander joints
    (legs on the landing pad from step 0; broadphase on in the forward)."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.lunar_case(8, 12, seed=0)
    ll = pa.LunarLander(batch=8)
    _, ret, ga, gd, _ = _gpu_rollout(torch, case, None, stages=pa._ffi.STAGES_LUNAR | pa._ffi.STAGE_BROADPHASE,
                                     world=ll.world)
    _check_grad_vs_oracle(case, ret, ga, gd)
    assert np.abs(gd).max() > 1.0


def test_rollout_grad_lunar_settled_full_size_sampled(torch_cuda):
    """The bench's grad_lunar workload at full size: 4096 LunarLanders settled
    on the terrain (2560 driver steps), a 32-step rollout with the lander's
    per-step dv, 8 envs sampled across the batch against the VJP oracle
    started from the same GPU state and keys (returns bit-exact)."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    B, T = 4096, 32
    ll = pa.LunarLander(batch=B)
    st = pa._ffi.STAGES_LUNAR | pa._ffi.STAGE_BROADPHASE
    for _ in range(40):
        ll.world.step(64, 1e-2, st)
    S0 = ll.world.dyn.permute(2, 0, 1).contiguous().cpu().numpy()
    keys = ll.world.keys.cpu().numpy().view(np.uint32)
    rng = np.random.default_rng(3)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(24, np.float32)
    w[0] = 1.0
    acts = torch.tensor(actions, device="cuda")
    ret, saved = pa.rollout_forward(ll.world, acts, 0, w, stages=st)
    ga, gd = pa.rollout_backward(ll.world, saved, want_dyn0=True)
    _check_tape_vs_replay(pa, ll.world, saved, ga, gd)
    ret, ga, gd = ret.cpu().numpy(), ga.cpu().numpy(), gd.cpu().numpy()
    assert np.isfinite(ga).all(axis=(0, 2)).mean() > 0.9
    envs = list(range(0, B, B // 8))
    case = dict(make=lambda: P.lunar_lander_bodies(prng.PRNGKey(0)), S0=S0[envs], keys=keys[envs],
                actions=actions[:, envs], w=w, ab=0, step=P.lunar_lander_step, tol=GC.POLYGON_TOL,
                name="lunar_settled_4096")
    _check_grad_vs_oracle(case, ret[envs], ga[:, envs], gd[:, :, envs])


def test_rollout_grad_polygon_box_vs_oracle(torch_cuda):
    """AABB x polygon and polygon x polygon contacts of rotating polygons."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.poly_box_case(8, 10, seed=0)
    _, ret, ga, gd, _ = _gpu_rollout(torch, case, _pa_bodies(pa, case["make"]()))
    _check_grad_vs_oracle(case, ret, ga, gd)


def test_rollout_grad_ball_on_polygons_vs_oracle(torch_cuda):
    """Gradients through circle x polygon contacts (cotix/_contacts.py:157-202):
    GJK + EPA with the circle's direction-dependent support, differentiated
    through every point of the chain (cx::circle_poly_vjp), against the
    torch-f32 VJP oracle (checked against finite differences in
    tests/test_grad_cpu.py); tape and re-play backwards bit for bit."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.ball_poly_case(16, 12, seed=1)
    _, ret, ga, gd, _ = _gpu_rollout(torch, case, _pa_bodies(pa, case["make"]()))
    _check_grad_vs_oracle(case, ret, ga, gd)
    assert np.isfinite(ga).all() and np.abs(ga).max() > 0.1


def test_rollout_grad_quad_row_vs_oracle(torch_cuda):
    """Nine polygons of one contact type: the contact VJPs inside phase G, at
    the scene's default tiling (2 envs per wave: its tile exceeds the LDS at
    4, so cotix_scene_create picks 2)."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.quad_row_case(8, 6, seed=0)
    w, ret, ga, gd, _ = _gpu_rollout(torch, case, _pa_bodies(pa, case["make"]()))
    assert w.scene.variant()["envs_per_wave"] == 2
    _check_grad_vs_oracle(case, ret, ga, gd)


def test_rollout_grad_robocup_vs_oracle(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    case = GC.robocup_case(16, 8)
    _, ret, ga, _, _ = _gpu_rollout(torch, case, pa.scenarios.robocup_bodies())
    orc = GC.oracle(case)
    for e in orc:
        r, oga, _ = orc[e]
        assert (np.isnan(ret[e]) and np.isnan(r)) or np.float32(ret[e]).view(np.uint32) == np.float32(r).view(
            np.uint32), (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d %s" % (e, msg)


def test_rollout_config5_full_size_vs_vjp_oracle(torch_cuda):
    """BASELINE config 5 at full size (4096 envs x 64 steps) checked
    independently of the kernel's host emulation, against the torch-f32 VJP
    oracle of the reference step (oracle/cotix_oracle/grad.py, itself checked
    against finite differences in tests/test_grad_cpu.py).  On this scene most
    envs' gradients are NaN (the reference's NaN at step 1 and its error_if
    trip), so the sample is taken from the GPU run's own split: 32 envs spread
    over the FINITE-gradient set (every entry compared at GC.ANALYTIC_TOL:
    rtol 1e-5 elementwise + 1e-7 * max|want|) and 32 over the rest (the NaN
    pattern compared exactly).  Return bit for bit in all 64.  Prints the floor
    each sampled block needed."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    B, T = 4096, 64
    case = GC.robocup_case(B, T)
    _, ret, ga, _, _ = _gpu_rollout(torch, case, pa.scenarios.robocup_bodies())
    fin = np.isfinite(ga).all(axis=(0, 2))  # ga [T, B, 2]
    fin_envs, nan_envs = np.flatnonzero(fin), np.flatnonzero(~fin)
    assert len(fin_envs) >= 32 and len(nan_envs) >= 32, (len(fin_envs), len(nan_envs))
    pick = lambda ids: [int(ids[i]) for i in np.linspace(0, len(ids) - 1, 32).round().astype(int)]  # noqa: E731
    sf, sn = pick(fin_envs), pick(nan_envs)
    orc = GC.oracle_parallel(case, sf + sn)
    need = 0.0
    for e in sf + sn:
        r, oga, _ = orc[e]
        assert (np.isnan(ret[e]) and np.isnan(r)) or np.float32(ret[e]).view(np.uint32) == np.float32(r).view(
            np.uint32), (e, ret[e], r)
        ok, msg = GC.close(ga[:, e], oga, case["tol"], case["name"])
        assert ok, "env %d %s" % (e, msg)
        if e in sf:
            assert np.isfinite(oga).all(), "env %d: finite on the GPU, not in the oracle" % e
            want = oga.astype(np.float64)
            m = np.abs(want).max()
            excess = np.abs(ga[:, e].astype(np.float64) - want) - 1e-5 * np.abs(want)
            need = max(need, float(excess.max()) / m if m > 0 else 0.0)
    print("config-5 full size: %d finite / %d NaN-pattern envs compared; floor needed at rtol 1e-5: %.3g"
          % (len(sf), len(sn), max(need, 0.0)))


def test_rollout_config5_full_size_vs_emulation(torch_cuda):
    """BASELINE config 5 at full size (4096 envs x 64 steps): forward state,
    return and every gradient equal the host emulation of the same kernel
    code bit for bit (the emulation is pinned to the oracle by
    tests/test_grad_cpu.py); then autograd through pa.differentiable_rollout."""
    torch = torch_cuda
    import parallax_amd as pa
    import grad_cases as GC
    sys_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu")
    import sys
    sys.path.insert(0, sys_path)
    import emu
    lib = emu.load()
    B, T = 4096, 64
    case = GC.robocup_case(B, T)
    w, ret, ga, gd, saved = _gpu_rollout(torch, case, pa.scenarios.robocup_bodies())
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    keys = np.array(case["keys"], np.uint32, copy=True)
    err = np.zeros(B, np.uint32)
    eret, esd, esk, etape = emu.rollout(lib, h, dyn, keys, err, geom, 0, 21, case["actions"], case["ab"], case["w"])
    ega, egd = emu.rollout_backward(lib, h, esd, esk, geom, 0, 21, case["actions"], case["ab"], case["w"],
                                    tape=etape)
    assert same_f32(w.dyn.cpu().numpy(), dyn)
    assert same_f32(saved["dyn"].cpu().numpy(), esd)
    assert same_f32(ret, eret)
    assert same_f32(ga, ega), diff_report(ga, ega)
    assert same_f32(gd, egd), diff_report(gd, egd)
    fin = np.isfinite(ga).all(axis=(0, 2))
    assert fin.any()
    # autograd surface: d(sum_env g_env * R_env)/d action = g_env * dR_env/d action
    w2 = pa.World(pa.scenarios.robocup_bodies(), B, "cuda", torch.tensor(u32_to_i32(case["keys"]), device="cuda"))
    w2.dyn.copy_(torch.tensor(case["S0"], device="cuda").permute(1, 2, 0))
    acts = torch.tensor(case["actions"], device="cuda", requires_grad=True)
    R = pa.differentiable_rollout(w2, acts, case["ab"], case["w"])
    g = torch.linspace(0.5, 1.5, B, device="cuda")
    (R[torch.isfinite(R)] * g[torch.isfinite(R)]).sum().backward()
    got = acts.grad.cpu().numpy()[:, fin]
    want = (ga * g.cpu().numpy()[None, :, None])[:, fin]
    assert np.allclose(got, want, rtol=1e-6, atol=0)


# ---------------------------------------------------------------------------
# AbstractEnvironment.eval (cotix/_envs.py:37-132) over the fused kernel
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("scene", ["box", "robocup"])
def test_eval_physics_world_vs_oracle(torch_cuda, scene):
    torch = torch_cuda
    import parallax_amd as pa
    from parallax_amd import envs as E
    import eval_cases as EC
    import grad_cases as GC
    from cotix_oracle import envs as OE
    B = 8
    case = GC.box_case(B, 1, seed=5) if scene == "box" else GC.robocup_case(B, 1)
    ab = case["ab"]
    if scene == "box":
        case["S0"][1, ab, 0] = 1.5
        bodies = _pa_bodies(pa, case["make"]())
    else:
        bodies = pa.scenarios.robocup_bodies()
    w = pa.World(bodies, B, "cuda")
    state = E.WorldState(torch.tensor(case["S0"], device="cuda").permute(1, 2, 0).contiguous(),
                         torch.tensor(u32_to_i32(case["keys"]), device="cuda"),
                         torch.zeros(B, dtype=torch.int32, device="cuda"))
    env = E.AbstractEnvironment(E.PhysicsWorld(w), state, EC.PDControl(ab), EC.XJudge(ab))
    out, reward = env.eval(0.6, 3, 10)
    torch.cuda.synchronize()
    for e in range(B):
        ob = case["make"]()
        for b, row in zip(ob, case["S0"][e]):
            b.set_dyn(row)
        (fb, fk), orew = OE.eval_env(case["step"], (ob, np.asarray(case["keys"][e], np.uint32)), EC.OraclePD(ab),
                                     EC.OracleX(ab), 0.6, 3, 10, GC.D0, ab)
        want = np.array([b.dyn() for b in fb], np.float32)
        assert same_f32(out.state.dyn[:, :, e].cpu().numpy(), want), e
        assert np.array_equal(out.state.keys[e].cpu().numpy().view(np.uint32), fk)
        assert same_f32(reward[e:e + 1].cpu().numpy(), np.array([orew], np.float32)), (e, reward[e], orew)


# ---------------------------------------------------------------------------
# body-level operators (UniversalShape, cotix/_universal_shape.py:87-132)
# ---------------------------------------------------------------------------
def test_body_operators_vs_oracle(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    import body_cases as BC
    import grad_cases as GC
    from cotix_oracle import universal as U
    B = 256
    make = lambda: BC.bodies(3)  # noqa: E731
    obodies = make()
    bodies = []
    for b in obodies:
        parts = []
        for p in b.parts:
            if p.kind == "Circle":
                parts.append(pa.Circle(p.radius, list(p.position)))
            elif p.kind == "AABB":
                parts.append(pa.AABB(list(p.lower), list(p.upper)))
            else:
                parts.append(pa.Polygon([list(v) for v in p.vertices_]))
        bodies.append(pa.AnyBody(shape=pa.UniversalShape(*parts), mass=1.0, inertia=1.0))
    w = pa.World(bodies, B, "cuda")
    dyn = BC.states(B, seed=11)
    w.dyn.copy_(torch.tensor(dyn, device="cuda"))
    for (i, j) in [(0, 1), (1, 2), (2, 0)]:
        col, pen = w.penetrates_with(i, j)
        col, pen = col.cpu().numpy(), pen.cpu().numpy()
        pc = w.possibly_collides_with(i, j).cpu().numpy()
        for e in range(B):
            bi, bj = BC.oracle_body(make, dyn, e, i), BC.oracle_body(make, dyn, e, j)
            ok, p = U.penetrates_with(bi, bj, GC.D0)
            assert bool(col[e]) == ok and same_f32(pen[e], np.array(p, np.float32)), (i, j, e)
            (ai, _), (aj, _) = U.body_aabb(bi), U.body_aabb(bj)
            sep = ai[3] <= aj[1] or ai[2] <= aj[0] or ai[1] >= aj[3] or ai[0] >= aj[2]
            assert bool(pc[e]) == (not sep), (i, j, e)
            # (no "narrowphase implies broadphase" check: through the reference's
            # wrap_local_support a rotated body's support is not its true extreme
            # point, so neither operator bounds the other for rotated bodies)


# ---------------------------------------------------------------------------
# observation / render export and the state contract
# ---------------------------------------------------------------------------
def test_observe_and_check_state(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=1000, device="cuda", perturb=True), autoreset=True)
    env.reset()
    env.step(7)
    obs = env.observation()
    torch.cuda.synchronize()
    assert obs.is_contiguous() and tuple(obs.shape) == (1000, 5, 6)
    assert same_f32(obs.cpu().numpy(), env.world.dyn.permute(2, 0, 1).cpu().numpy())
    env.reset()  # a finite state (stepped RoboCup states hold NaN velocities: the reference's error_if trips)
    w = env.world
    w.err.zero_()
    w.dyn[1, 3, 17] = float("nan")
    w.dyn[4, 0, 999] = float("inf")
    w.err[5] = 1
    w.check_state()
    want = np.zeros(1000, np.int32)
    want[5] = 1
    want[[17, 999]] |= pa._ffi.ERR_STATE_NONFINITE
    assert np.array_equal(w.err.cpu().numpy(), want)


@pytest.mark.parametrize("scene", ["robocup", "lunar"])
def test_render_draw_vs_reference(torch_cuda, scene):
    """env.draw(painter) through the render kernel == the reference's Painter
    call sequence (oracle restatement), coordinates bit for bit."""
    torch = torch_cuda
    import parallax_amd as pa
    import parallax_amd.render as R
    from cotix_oracle import physics as P
    from cotix_oracle import render as OR
    from cotix_oracle import prng
    import test_render_contracts_cpu as T
    if scene == "robocup":
        sc = pa.RoboCupEnv(batch=64, device="cuda", perturb=True)
        sc.world.step(5, 1e-2, sc.stages)
        mk = lambda e: P.robocup_bodies()  # noqa: E731
        draw = OR.robocup_draw
    else:
        keys = pa.random.split(pa.random.PRNGKey(0, "cuda"), 64).contiguous()
        sc = pa.LunarLander(key=keys, batch=64, device="cuda")
        sc.world.dyn[:3, 4] += torch.linspace(-1.0, 1.0, 64, device="cuda")  # rotated landers
        tk = prng.split(prng.PRNGKey(0), 64)
        mk = lambda e: P.lunar_lander_bodies(tk[e])  # noqa: E731
        draw = OR.lunar_lander_draw
    prims = R.render(sc.world)
    dyn = sc.world.dyn.cpu().numpy()
    for e in (0, 1, 31, 63):
        bodies = mk(e)
        for i, b in enumerate(bodies):
            b.set_dyn(dyn[i, :, e])
        p = R.RecordingPainter()
        sc.draw(p, env=e, prims=prims)
        T._same_calls(p.calls, draw(bodies))


# ---------------------------------------------------------------------------
# ragged batches: B not a multiple of the envs-per-wave tile (4), a wave
# whose tail lanes hold no env, and B = 0 / negative sizes through the C-ABI
# ---------------------------------------------------------------------------
def _subset_check(torch, make, big, stages, T, sizes):
    """Each env's result is independent of its batch: a world of
    the first b envs must reproduce those envs of the big run bit for bit,
    and must not write past B (keys/err live in larger sentinel buffers)."""
    init = big.dyn.clone()
    keys0 = big.keys.clone()
    big.step(T, 1e-2, stages)
    torch.cuda.synchronize()
    for b in sizes:
        w = make(b)
        w.dyn.copy_(init[:, :, :b])
        kbuf = torch.full((b + 8, 2), 0x5A5A5A5A, dtype=keys0.dtype, device="cuda")
        kbuf[:b] = keys0[:b]
        ebuf = torch.full((b + 8,), 0x5A5A5A5A, dtype=big.err.dtype, device="cuda")
        ebuf[:b] = 0
        dyn = w.dyn.clone()
        w.step_state(dyn, kbuf[:b], ebuf[:b], T, 1e-2, stages)
        torch.cuda.synchronize()
        assert same_f32(dyn.cpu().numpy(), big.dyn[:, :, :b].cpu().numpy()), "B=%d" % b
        assert torch.equal(kbuf[:b], big.keys[:b]) and torch.equal(ebuf[:b], big.err[:b]), "B=%d" % b
        assert bool((kbuf[b:] == 0x5A5A5A5A).all()) and bool((ebuf[b:] == 0x5A5A5A5A).all()), "B=%d wrote past B" % b


@pytest.mark.parametrize("ew", ["1", "2", "4", "8"])
def test_ragged_batches_robocup(torch_cuda, ew):
    torch = torch_cuda
    import parallax_amd as pa
    env = pa.RoboCupEnv(batch=64, device="cuda", perturb=True)
    env.world.set_variant(int(ew))
    keys = env.world.keys.clone()
    _subset_check(torch, lambda b: pa.RoboCupEnv(batch=b, device="cuda", keys=keys[:b].clone()).world.set_variant(
        int(ew)), env.world, env.stages, 8, [1, 3, 5, 13, 63])


def test_ragged_batches_lunar(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import prng
    tkeys = torch.tensor(u32_to_i32(prng.split(prng.PRNGKey(0), 64)), device="cuda")
    ll = pa.LunarLander(key=tkeys, batch=64, device="cuda")
    for i in range(3):  # drop every other lander onto the ground so GJK/EPA contacts fire
        ll.world.dyn[i, 1, ::2] -= 6.3
        ll.world.dyn[i, 3, ::2] = -0.3
    ck = ll.world.keys.clone()
    _subset_check(torch, lambda b: pa.LunarLander(key=tkeys[:b].clone(), batch=b, device="cuda",
                                                  collider_keys=ck[:b].clone()).world,
                  ll.world, ll.stages, 4, [1, 2, 7, 33])


def test_empty_and_negative_sizes(torch_cuda):
    torch = torch_cuda
    import ctypes
    import parallax_amd as pa
    from parallax_amd import _ffi
    env = pa.RoboCupEnv(batch=4, device="cuda", perturb=True)
    w = env.world
    before = w.dyn.clone()
    s = _ffi.stream_ptr(w.device)
    args = lambda B, n: (w.scene.handle, _ffi.ptr(w.dyn), _ffi.ptr(w.keys), _ffi.ptr(w.err), _ffi.ptr(w.geom),
                         w.geom_stride, B, n, ctypes.c_float(1e-2), int(env.stages), None, 0, s)
    assert _ffi.lib.cotix_step(*args(0, 5)) == 0
    assert _ffi.lib.cotix_step(*args(4, 0)) == 0
    torch.cuda.synchronize()
    assert torch.equal(w.dyn, before)
    assert _ffi.lib.cotix_step(*args(-1, 1)) < 0
    assert b"negative" in _ffi.lib.cotix_last_error()
    assert _ffi.lib.cotix_step(*args(4, -1)) < 0


def test_rank_shards_concatenate_to_single_run(torch_cuda):
    """SURVEY 8(e) on the GPU: each of 4 ranks BUILDS its shard from its global
    env ids with bench.py's constructor (RoboCupEnv(env_offset=r*n,
    total_envs=B): keys and ball perturbations sliced from one global split,
    only global env 0 unperturbed) and steps it; the shards concatenate to the
    single-device run bit for bit, collider choices included."""
    torch = torch_cuda
    import parallax_amd as pa
    B, R, T = 256, 4, 8
    full = pa.RoboCupEnv(batch=B, device="cuda", perturb=True)
    ftr = {}
    full.world.step(T, 1e-2, full.stages, trace=ftr)
    parts = []
    n = B // R
    for r in range(R):
        sh = pa.RoboCupEnv(batch=n, device="cuda", perturb=True, env_offset=r * n, total_envs=B)
        tr = {}
        sh.world.step(T, 1e-2, sh.stages, trace=tr)
        parts.append((sh.world.dyn, sh.world.keys, sh.world.err, tr["chosen"], tr["cells"]))
    torch.cuda.synchronize()
    assert same_f32(torch.cat([p[0] for p in parts], 2).cpu().numpy(), full.world.dyn.cpu().numpy())
    assert torch.equal(torch.cat([p[1] for p in parts]), full.world.keys)
    assert torch.equal(torch.cat([p[2] for p in parts]), full.world.err)
    assert torch.equal(torch.cat([p[3] for p in parts], 2), ftr["chosen"])
    assert torch.equal(torch.cat([p[4] for p in parts], 3), ftr["cells"])
    # rank 1..3 shards are not copies of rank 0's (the bug bench.py once had)
    assert not torch.equal(parts[0][0][4], parts[1][0][4])


def test_config4_global_size_shards_concatenate(torch_cuda):
    """BASELINE config 4 at its full global size on one GPU: the 8 rank shards
    of 8192 envs, each BUILT from its global env ids 0..65535 as bench.py's
    rank r does (RoboCupEnv(env_offset=8192 r, total_envs=65536), restarts on
    the error trip), stepped 2 x 8 fused steps, concatenate to ONE
    65,536-env launch bit for bit: state, keys, errors, restart counts and
    every collider choice (chosen partner per body, winning candidate per
    cell) of the second launch."""
    torch = torch_cuda
    import parallax_amd as pa
    N, R, T = 65536, 8, 8
    n = N // R

    def run(env):
        resets = torch.zeros(env.world.B, dtype=torch.int32, device="cuda")
        env.world.step(T, 1e-2, env.stages, dyn_reset=env.dyn_reset, resets=resets)
        tr = {}
        env.world.step(T, 1e-2, env.stages, dyn_reset=env.dyn_reset, resets=resets, trace=tr)
        return env.world.dyn, env.world.keys, env.world.err, resets, tr["chosen"], tr["cells"]

    full = run(pa.RoboCupEnv(batch=N, device="cuda", perturb=True))
    shards = [run(pa.RoboCupEnv(batch=n, device="cuda", perturb=True, env_offset=r * n, total_envs=N))
              for r in range(R)]
    torch.cuda.synchronize()
    for q, cat_dim in enumerate((2, 0, 0, 0, 2, 3)):
        got = torch.cat([sh[q] for sh in shards], cat_dim)
        assert torch.equal(got.view(torch.int32), full[q].view(torch.int32)), q
    assert int(full[3].sum()) > N  # the restarts ran (most envs trip within 2 steps)


def test_contracts_and_check_state_vs_oracle(torch_cuda):
    """Row f4 as a parity row: the device state check (cotix_check_state, the
    invariant "NaN or invalid value encountered", cotix/_design_by_contract.py:
    80-107) and the contract wrappers applied to device tensors
    (parallax_amd.contracts: error_if / pre_condition / post_condition /
    class_invariant, :13-107) against the oracle's scalar restatement
    (oracle/cotix_oracle/contracts.py), env by env, on a ragged batch with
    NaN, +-inf, -0, denormal and extreme finite words."""
    torch = torch_cuda
    import parallax_amd as pa
    from parallax_amd import contracts as C
    from parallax_amd.envs import WorldState
    from cotix_oracle import contracts as OC
    rng = np.random.default_rng(5)
    B = 4099
    dyn = (rng.normal(size=(5, 6, B)) * 10).astype(np.float32)
    special = np.array([np.nan, np.inf, -np.inf, -0.0, 1e-45, 3.4e38, -3.4e38, 1.2e-38], np.float32)
    pos = rng.integers(0, dyn.size, 400)
    dyn.reshape(-1)[pos] = special[rng.integers(0, special.size, pos.size)]
    err0 = rng.integers(0, 4, B).astype(np.int32)
    w = pa.World(pa.scenarios.robocup_bodies(), B, "cuda")
    w.dyn.copy_(torch.tensor(dyn))
    w.err.copy_(torch.tensor(err0))
    w.check_state()
    want = OC.check_state(dyn, err0)
    assert 0 < int((want & OC.ERR_STATE_NONFINITE).astype(bool).sum()) < B
    assert np.array_equal(w.err.cpu().numpy().astype(np.int64), want)

    # error_if on a device WorldState
    pred = rng.random(B) < 0.3
    st = C.error_if(WorldState(w.dyn.clone(), w.keys.clone(), torch.tensor(err0, device="cuda")),
                    torch.tensor(pred, device="cuda"))
    gd, ge = st.dyn.cpu().numpy(), st.err.cpu().numpy()
    for e in range(B):
        wd, we = OC.env_state_error_if(dyn[:, :, e].reshape(-1).tolist(), int(err0[e]), bool(pred[e]))
        assert same_f32(gd[:, :, e].reshape(-1), np.array(wd, np.float32)) and ge[e] == we, e

    # pre / post conditions on device tensors, per env
    x = rng.normal(size=B).astype(np.float32)
    y = rng.normal(size=B).astype(np.float32)
    xt, yt = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    got = C.pre_condition(lambda a, b: a > 0)(lambda a, b: a + b)(xt, yt).cpu().numpy()
    want = np.array([OC.pre_condition(lambda a, b: a > 0, lambda a, b: a + b, x[e], y[e]) for e in range(B)],
                    np.float32)
    assert same_f32(got, want)
    got = C.post_condition(lambda r, a: r > a, provide_input=True)(lambda a: a * np.float32(1.5) - 1)(xt)
    want = np.array([OC.post_condition(lambda r, a: r > a, lambda a: a * np.float32(1.5) - np.float32(1), x[e],
                                       provide_input=True) for e in range(B)], np.float32)
    assert same_f32(got.cpu().numpy(), want)

    # class_invariant: the guard fires where __invariant__() is true
    @C.class_invariant
    class Probe:
        def __init__(self, v):
            self.v = v

        def __invariant__(self):
            return self.v < 0

        def value(self):
            return self.v * 2

    got = Probe(xt.clone()).value().cpu().numpy()
    want = np.array([np.float32(np.nan) if OC.class_invariant_fires(x[e] < 0) else x[e] * np.float32(2)
                     for e in range(B)], np.float32)
    assert same_f32(got, want)


# ---------------------------------------------------------------------------
# named regressions of the two hipcc 7.2 miscompiles found this far
# (DESIGN.md section 8); both are also covered indirectly by the fixtures
# ---------------------------------------------------------------------------
def test_regression_hipcc_support_p4xp6(torch_cuda):
    """A guarded, branchy unrolled argmax in the polygon support function was
    miscompiled at -O2/-O3: 38 of the P4 x P6 fixture pairs lost their
    contact.  The 400 P4 x P6 pairs of the poly_poly fixture: every contact
    bit-exact and the count of contacts equal to the oracle's."""
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a, b = g["poly_poly_a"], g["poly_poly_b"]
    sel = (a[:, 1] == 4) & (b[:, 1] == 6)
    assert sel.sum() >= 400
    info, _ = pa.run_contacts(int(g["poly_poly_fn"]), torch.tensor(a[sel], device="cuda"),
                              torch.tensor(b[sel], device="cuda"))
    got = torch.cat([info.penetration_vector, info.contact_point], 1).cpu().numpy()
    want = g["poly_poly_out"][sel]
    assert same_f32(got, want), diff_report(got, want)
    assert (~np.isnan(got[:, 2])).sum() == (~np.isnan(want[:, 2])).sum() > 0


@pytest.mark.parametrize("ew", ["1", "2", "4", "8"])
def test_regression_hipcc_mixed_kind_transform(torch_cuda, cport_lib, ew):
    """A divergent circle / AABB tail of the part transform (phase T) faulted
    (aperture violation: the circle lanes used an address only the AABB lanes
    had defined).  RoboCup's parts mix a circle with AABBs; every envs-per-
    wave tiling puts different kind mixes in one wave.  64 perturbed envs, 6
    fused steps with restarts, against the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=64, device="cuda", perturb=True), autoreset=True)
    env.world.set_variant(int(ew))
    env.reset()
    dyn = np.ascontiguousarray(env.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(env.world.keys.cpu().numpy().view(np.uint32))
    _robocup_vs_cport(torch, pa, cport, lib, env, dyn, keys, 1, 6)


@pytest.mark.parametrize("scene", ["robocup", "lunar", "box"])
def test_specialized_kernel_equals_generic(torch_cuda, scene):
    """The scene-specialized instantiations (the two reference scenes' headers
    as compile-time constants, cxk::SPEC_*, at 4 and 2 envs per wave) and the
    generic kernel (specialize=0) give bit-identical state, keys, error bits,
    restarts and collider traces."""
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import prng
    outs = []
    for ew, spec in ((4, True), (4, False), (2, True)):
        if scene == "robocup":
            env = pa.BatchedEnv(pa.RoboCupEnv(batch=1000, device="cuda", perturb=True), autoreset=True)
        elif scene == "box":
            if ew == 2:
                continue  # (the box world's specialization: the 4-env tiling)
            env = pa.BatchedEnv(pa.BoxWorld(batch=1000, device="cuda"), autoreset=True)
        else:
            tk = torch.tensor(u32_to_i32(prng.split(prng.PRNGKey(0), 1000)), device="cuda")
            env = pa.BatchedEnv(pa.LunarLander(key=tk, batch=1000, device="cuda"), autoreset=True)
            env.scenario.dyn_reset[:3, 1, ::2] -= 6.3  # half of the landers start on the ground
        env.world.set_variant(ew, spec)
        assert env.world.scene.variant() == {"envs_per_wave": ew, "specialization": scene if spec else "generic"}
        env.reset()
        trc = {}
        env.step(24, trace=trc)
        torch.cuda.synchronize()
        outs.append([env.world.dyn.cpu().numpy(), env.world.keys.cpu().numpy(), env.world.err.cpu().numpy(),
                     env.resets.cpu().numpy(), trc["chosen"].cpu().numpy(), trc["cells"].cpu().numpy()])
    for o in outs[1:]:
        assert same_f32(outs[0][0], o[0])
        for g, w in zip(outs[0][1:], o[1:]):
            assert np.array_equal(g, w)
    assert (outs[0][5] >= 0).any()


def _world_from_oracle(pa, torch, bodies, B, keys):
    """A World of B envs of the oracle's bodies (local geometry as the oracle
    holds it: polygons presorted)."""
    kinds = {"Polygon": pa.Polygon, "Polygon3": pa.Polygon3, "Polygon4": pa.Polygon4, "Polygon5": pa.Polygon5,
             "Polygon6": pa.Polygon6}
    out = []
    for b in bodies:
        parts = []
        for p in b.parts:
            if p.kind == "AABB":
                parts.append(pa.AABB(list(p.lower), list(p.upper)))
            elif p.kind == "Circle":
                parts.append(pa.Circle(p.radius, list(p.position)))
            else:
                parts.append(kinds[p.kind]([list(v) for v in p.vertices_], presorted=True))
        out.append(pa.AnyBody(shape=pa.UniversalShape(*parts), mass=b.mass, inertia=b.inertia,
                              position=list(b.position), velocity=list(b.velocity), angle=b.angle,
                              angular_velocity=b.angular_velocity, elasticity=b.elasticity,
                              friction_coefficient=b.friction_coefficient))
    return pa.World(out, B, "cuda", torch.tensor(u32_to_i32(keys), device="cuda"))


@pytest.mark.parametrize("scene", ["aabb_poly", "aabb_circle_poly", "straddle", "straddle_ew1", "octagons9",
                                   "octagons12", "octagons15", "polygon20"])
def test_generic_polygon_scenes_vs_cport(torch_cuda, cport_lib, scene):
    """The generic step programs on the GPU (cxk::launch_fnset: polygon-only
    GJK/EPA for the straddling-part scene, AABB x polygon, circle x polygon)
    against the C port: 512 envs x 24 steps, state, keys, errors and every
    contact choice.  straddle_ew1: one env per wave, where the static floor
    straddles phase T's first two vertex-item chunks.  octagons9: nine
    octagon bodies, whose tile fits the LDS at one env per wave only -- the
    tiling the library picks at scene creation.  octagons12 / octagons15 /
    polygon20 (20 polygon parts over 5 bodies): tiles that fit only in
    workgroups of fewer than four waves (cotix_scene_waves_per_group)."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    import scene_cases
    if scene.startswith("octagons"):
        bodies = scene_cases.octagon_row(int(scene[8:]))
    elif scene == "polygon20":
        bodies = scene_cases.polygon20()
    else:
        bodies = scene_cases.straddle_scene(4.0) if scene.startswith("straddle") else scene_cases.mixed_scene(
            scene == "aabb_circle_poly")
    B, T = 512, 24
    keys = np.ascontiguousarray(np.stack([np.arange(B) + 3, np.arange(B) * 5 + 1], 1).astype(np.uint32))
    w = _world_from_oracle(pa, torch, bodies, B, keys)
    if scene == "straddle_ew1":
        w.set_variant(1)
    if scene == "octagons9":
        assert w.scene.variant()["envs_per_wave"] == 1 and w.scene.waves_per_group() == 4
    if scene in ("octagons12", "octagons15", "polygon20"):
        assert w.scene.variant()["envs_per_wave"] == 1 and w.scene.waves_per_group() in (1, 2)
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[0, 0, :] += np.linspace(-0.6, 0.6, B).astype(np.float32)
    w.set_dyn(torch.tensor(dyn, device="cuda"))
    err = np.zeros(B, np.uint32)
    trc = {}
    w.step(T, 1e-2, pa._ffi.STAGES_ROBOCUP, trace=trc)
    sc = cport.Scene(lib, bodies)
    wch, wcl = sc.step_ex(dyn, keys, err, T, cport.STAGES_ROBOCUP, trace=True, nthreads=16)
    torch.cuda.synchronize()
    assert (wcl >= 0).sum() > B
    got = w.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(w.err.cpu().numpy().view(np.uint32), err)
    assert np.array_equal(trc["chosen"].cpu().numpy(), wch)
    assert np.array_equal(trc["cells"].cpu().numpy(), wcl)
