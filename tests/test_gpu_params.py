"""GPU parity of the scene parameter block (include/cotix_amd.h cotix_params)
through the C-ABI: the partitionable threefry layout and a non-default
constant set (tests/param_sets.py) bit-exact against the oracle's golden
fixtures and the C port at the BASELINE sizes -- state, keys, error bits and
every contact choice (j* per body, winning candidate per all_contacts cell,
cotix/_colliders.py:208-295) -- plus the GJK / EPA operators
(cotix/_collisions.py:277-329) against their fixtures."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, HERE)

from param_sets import PARAM_SETS, host_params, oracle_params  # noqa: E402
from test_gpu_parity import _check_trace, diff_report, same_f32, u32_to_i32  # noqa: E402

VARIANTS = ["_part", "_alt"]
ALL = ["", "_part", "_alt"]


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


def test_prng_kernels_partitionable(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "prng_part.npz"))
    keys = torch.tensor(u32_to_i32(g["keys"][:16]), device="cuda")
    sp = pa.random.split(keys, 5, "partitionable").cpu().numpy().view(np.uint32)
    assert np.array_equal(sp, g["splits"])
    assert same_f32(pa.random.uniform(keys, 7, -3.0, 2.0, "partitionable").cpu().numpy(), g["uniform7"])
    assert same_f32(pa.random.uniform(keys, None, 4.0, 8.0, "partitionable").cpu().numpy(), g["uniform1"])
    # published (JAX >= 0.5 documentation): split(key(0)), uniform(key(0))
    k0 = pa.random.PRNGKey(0, "cuda")
    assert pa.random.split(k0, 2, "partitionable").cpu().numpy().view(np.uint32).tolist() == [
        [1797259609, 2579123966], [928981903, 3453687069]]
    assert pa.random.uniform(k0, None, layout="partitionable").item() == np.float32(0.947667)
    # the legacy kernels are unchanged
    assert pa.random.split(k0).cpu().numpy().view(np.uint32).tolist() == [[4146024105, 967050713],
                                                                          [2718843009, 1272950319]]


@pytest.mark.parametrize("per_step", [True, False])
@pytest.mark.parametrize("suffix", VARIANTS)
def test_robocup_trace_params(torch_cuda, suffix, per_step):
    torch = torch_cuda
    import parallax_amd as pa
    tr = np.load(os.path.join(GOLD, "robocup_trace%s.npz" % suffix))
    T, B = tr["err"].shape
    env = pa.RoboCupEnv(batch=B, device="cuda", perturb=True, params=host_params(suffix))
    # the scenario draws its keys and perturbations in the block's layout
    assert np.array_equal(env.world.keys.cpu().numpy().view(np.uint32), tr["keys"][0]), "keys"
    assert same_f32(env.world.dyn.permute(2, 0, 1).cpu().numpy(), tr["dyn"][0]), "perturbed reset state"
    _check_trace(env.world, tr, env.stages, T, per_step)


@pytest.mark.parametrize("per_step", [True, False])
@pytest.mark.parametrize("suffix", VARIANTS)
def test_lunar_trace_params(torch_cuda, suffix, per_step):
    torch = torch_cuda
    import parallax_amd as pa
    tr = np.load(os.path.join(GOLD, "lunar_trace%s.npz" % suffix))
    T, B = tr["err"].shape
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tr["terrain_keys"]), device="cuda"), batch=B, device="cuda",
                        collider_keys=torch.tensor(u32_to_i32(tr["keys"][0]), device="cuda"),
                        params=host_params(suffix))
    ll.world.dyn.copy_(torch.tensor(tr["init"], device="cuda").permute(1, 2, 0))
    _check_trace(ll.world, tr, ll.stages, T, per_step)


@pytest.mark.parametrize("suffix", ALL)
def test_gjk_epa_operators(torch_cuda, suffix):
    """cotix_gjk (hit, simplex; NaN * simplex without a collision) and
    cotix_epa at 3, 11 and 48 iterations over polygon / AABB / circle pairs
    and degenerate inputs, bit-exact against the fixtures."""
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "gjk_epa%s.npz" % suffix))
    a = torch.tensor(g["a"], device="cuda")
    b = torch.tensor(g["b"], device="cuda")
    hit, sx = pa.check_for_collision_convex(a, b, host_params(suffix))
    assert np.array_equal(hit.cpu().numpy().astype(np.int32), g["hit"])
    assert same_f32(sx.cpu().numpy(), g["simplex"]), diff_report(sx.cpu().numpy(), g["simplex"])
    s = torch.tensor(g["simplex"], device="cuda")
    for it in (3, 11, 48):
        pen = pa.compute_penetration_vector_convex(a, b, s, it).cpu().numpy()
        assert same_f32(pen, g["pen%d" % it]), (it, diff_report(pen, g["pen%d" % it]))
    with pytest.raises(RuntimeError, match="iters"):
        pa.compute_penetration_vector_convex(a, b, s, 2)


@pytest.mark.parametrize("name", ["poly_poly", "aabb_poly", "circle_poly"])
def test_contacts_ex_alt_vs_cport(torch_cuda, cport_lib, name):
    """cotix_contacts_ex under the non-default block (GJK 1 step, EPA 3
    iterations, circle x polygon EPA 20) vs the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    cport, lib = cport_lib
    from cotix_oracle import params
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a, b = np.ascontiguousarray(g[name + "_a"]), np.ascontiguousarray(g[name + "_b"])
    n, fn = a.shape[0], int(g[name + "_fn"])
    kw = dict(PARAM_SETS["_alt"], epa_circle_iters=20)
    want = np.zeros((n, 4), np.float32)
    err = np.zeros(n, np.uint32)
    lib.oracle_contacts_ex(fn, n, cport._p(a), cport._p(b), cport._p(want), cport._p(err),
                           cport.params_ref(params.Params(**kw)))
    info, gerr = pa.run_contacts(fn, torch.tensor(a, device="cuda"), torch.tensor(b, device="cuda"), pa.Params(**kw))
    got = torch.cat([info.penetration_vector, info.contact_point], 1).cpu().numpy()
    assert same_f32(got, want), diff_report(got, want)
    assert np.array_equal(gerr.cpu().numpy().view(np.uint32), err)
    assert not same_f32(got, g[name + "_out"])  # the block changes the results


def test_resolve_operator_alt_baumgarte(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import params
    from cotix_oracle import physics as P
    rng = np.random.default_rng(31)
    n = 300
    d1 = rng.normal(size=(n, 6)).astype(np.float32)
    d2 = rng.normal(size=(n, 6)).astype(np.float32)
    p1 = np.abs(rng.normal(size=(n, 4))).astype(np.float32) + 0.1
    p2 = np.abs(rng.normal(size=(n, 4))).astype(np.float32) + 0.1
    c = rng.normal(size=(n, 4)).astype(np.float32)
    want1, want2 = d1.copy(), d2.copy()
    with params.use(oracle_params("_alt")):
        for k in range(n):
            b1 = P.Body([], *p1[k, :2], elasticity=p1[k, 2], friction_coefficient=p1[k, 3])
            b2 = P.Body([], *p2[k, :2], elasticity=p2[k, 2], friction_coefficient=p2[k, 3])
            b1.set_dyn(d1[k])
            b2.set_dyn(d2[k])
            P.resolve_collision(b1, b2, ((c[k, 0], c[k, 1]), (c[k, 2], c[k, 3])))
            want1[k], want2[k] = b1.dyn(), b2.dyn()
    t1, t2 = torch.tensor(d1, device="cuda"), torch.tensor(d2, device="cuda")
    pa.resolve_collision(t1, torch.tensor(p1, device="cuda"), t2, torch.tensor(p2, device="cuda"),
                         torch.tensor(c, device="cuda"), host_params("_alt"))
    assert same_f32(t1.cpu().numpy(), want1), diff_report(t1.cpu().numpy(), want1)
    assert same_f32(t2.cpu().numpy(), want2), diff_report(t2.cpu().numpy(), want2)


# ---------------------------------------------------------------------------
# BASELINE sizes, every env, under each block: HIP path vs the C port
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("suffix", VARIANTS)
def test_robocup_4096_params_vs_cport(torch_cuda, cport_lib, suffix):
    """The bench workload (4096 perturbed envs, restarts, ball actions) under
    the block: 2 launches x 16 fused steps, every env's state, keys, error
    bits, restarts and contact choices vs the C port under the same block."""
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    cport, lib = cport_lib
    B, T = 4096, 16
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True, params=host_params(suffix)),
                        autoreset=True)
    env.reset()
    dyn = np.ascontiguousarray(env.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(env.world.keys.cpu().numpy().view(np.uint32))
    reset = dyn.copy()
    err = np.zeros(B, np.uint32)
    resets = np.zeros(B, np.uint32)
    sc = cport.Scene(lib, P.robocup_bodies(), oracle_params(suffix))
    rng = np.random.default_rng(5)
    for q in range(2):
        act = np.ascontiguousarray((rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)) if q else None
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
    assert resets.sum() > 0 and (wcl >= 0).any()


@pytest.mark.parametrize("suffix", VARIANTS)
def test_lunar_4096_params_vs_cport(torch_cuda, cport_lib, suffix):
    """LunarLander config 2 size under the block: 4096 envs (a third dropped
    onto the terrain: GJK / EPA / contact points fire), 8 fused steps with the
    broadphase on, vs the C port."""
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import params
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    cport, lib = cport_lib
    B, T = 4096, 8
    with params.use(oracle_params(suffix)):
        tkeys = prng.split(prng.PRNGKey(0), B)
        bodies0 = P.lunar_lander_bodies(tkeys[0])
    ll = pa.LunarLander(key=torch.tensor(u32_to_i32(tkeys), device="cuda"), batch=B, device="cuda",
                        params=host_params(suffix))
    drop = torch.zeros(B, device="cuda")
    drop[::3] = 6.25
    for i in range(3):
        ll.world.dyn[i, 1] -= drop
        ll.world.dyn[i, 3] = torch.where(drop > 0, torch.tensor(-0.3, device="cuda"), ll.world.dyn[i, 3])
    dyn = np.ascontiguousarray(ll.world.dyn.cpu().numpy())
    keys = np.ascontiguousarray(ll.world.keys.cpu().numpy().view(np.uint32))
    geom = np.ascontiguousarray(ll.world.geom.cpu().numpy())
    with params.use(oracle_params(suffix)):  # the terrain of env 17 in the block's layout
        want_row = cport.Scene(lib, P.lunar_lander_bodies(tkeys[17])).geom
    assert same_f32(geom[17], want_row), "terrain"
    err = np.zeros(B, np.uint32)
    trc = {}
    ll.world.step(T, 1e-2, ll.stages, trace=trc)
    sc = cport.Scene(lib, bodies0, oracle_params(suffix))
    wch, wcl = sc.step_ex(dyn, keys, err, T, cport.STAGES_LUNAR, geom, trace=True, nthreads=16)
    torch.cuda.synchronize()
    got = ll.world.dyn.cpu().numpy()
    assert same_f32(got, dyn), diff_report(got, dyn)
    assert np.array_equal(ll.world.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(ll.world.err.cpu().numpy().view(np.uint32), err)
    assert (wcl >= 0).sum() > B
    assert np.array_equal(trc["chosen"].cpu().numpy(), wch)
    assert np.array_equal(trc["cells"].cpu().numpy(), wcl)


@pytest.mark.parametrize("suffix", ["", "_part"])
def test_gjk_initial_direction_and_key(torch_cuda, suffix):
    """cotix_gjk_ex: check_for_collision_convex with per-item
    initial_direction and key (cotix/_collisions.py:277-298) bit-exact against
    the oracle's fixture (tests/golden/gjk_dir*.npz); key=PRNGKey(1) and a
    NaN initial direction reproduce the default operator."""
    torch = torch_cuda
    import parallax_amd as pa
    g = np.load(os.path.join(GOLD, "gjk_dir%s.npz" % suffix))
    a = torch.tensor(g["a"], device="cuda")
    b = torch.tensor(g["b"], device="cuda")
    prm = host_params(suffix) if suffix else None
    hit, sx = pa.check_for_collision_convex(a, b, prm, initial_direction=torch.tensor(g["init"], device="cuda"),
                                            key=g["keys"])
    assert np.array_equal(hit.cpu().numpy().astype(np.int32), g["hit"])
    assert same_f32(sx.cpu().numpy(), g["simplex"]), diff_report(sx.cpu().numpy(), g["simplex"])
    h0, s0 = pa.check_for_collision_convex(a, b, prm)
    h1, s1 = pa.check_for_collision_convex(a, b, prm, initial_direction=[float("nan"), 0.0],
                                           key=np.array([0, 1], np.uint32))
    assert torch.equal(h0, h1) and same_f32(s0.cpu().numpy(), s1.cpu().numpy())
