"""The reference's own contact invariants, run on the HIP contact kernels
(cotix_contacts) at the reference's case counts.

``_test_with_seed`` / ``_test_contact_info`` (test/test_collisions.py:23-159)
check, for random shape pairs, that a non-NaN contact point lies in both
shapes, that moving shape a by the penetration vector resolves the contact
and -- in "heavy" mode, 1 case in 50 -- that no shorter move resolves it and
that the shapes touch afterwards.  The reference runs N = 10,000,000 light +
200,200 heavy circle x circle cases (:208-223) and 2,010,000 + 40,200
circle x AABB cases (:281-300, N_ratio 0.2); the same counts run here,
batched on the device (tests/contact_invariants.py), and every case must
pass, as the reference asserts.  The polygon invariants the reference skips
as "not implemented" (:403-462, small_eps 1e-3, N_ratio 0.1) run at their
counts too: the reference asserts nothing for them; here the three with
convex shapes must pass every case, the random-hexagon one (mostly
non-convex shapes) passes 66 %, and for all four the GPU verdict of every
sampled case must equal the CPU oracle's verdict on the same shapes
(tests/contact_props.py).
Random inputs follow the reference's distributions with torch's generator
(jax.random is not available here); the 10 literal circle x AABB cases of
:226-278 are checked heavily as written.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MAX_CALLS_PER_VMAP = 10_000
TESTS_PER_SCENARIO = 10_000_000


def counts(n_ratio):
    n = int(n_ratio * TESTS_PER_SCENARIO)
    batches = 1 + n // MAX_CALLS_PER_VMAP
    return batches * MAX_CALLS_PER_VMAP, batches * (MAX_CALLS_PER_VMAP // 50)


@pytest.fixture(scope="module")
def ci():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a visible GPU (torch.cuda.is_available() is False)")
    import contact_invariants
    return contact_invariants


def _f(fn):
    import parallax_amd as pa

    def f(a, b):
        info, _ = pa.run_contacts(fn, a, b)
        return info.penetration_vector, info.contact_point
    return f


def _oracle_f(fn):
    from cotix_oracle import geometry as G
    from cotix_oracle import prng
    d0 = prng.gjk_initial_direction()
    table = {1: lambda a, b, e: G.circle_vs_circle(a, b, e), 2: lambda a, b, e: G.circle_vs_aabb(a, b, e),
             3: lambda a, b, e: G.polygon_vs_polygon(a, b, d0, e), 4: lambda a, b, e: G.aabb_vs_polygon(a, b, d0, e)}

    def f(a, b):
        return table[fn](a, b, G.ErrorFlag())
    return f


def _run(ci, fn, gen_a, gen_b, n_ratio, small_eps, seed, chunk=2_000_000, chunk_heavy=40_000, sample=(0, 0)):
    """All light and heavy cases; returns (light fails, heavy fails, light n,
    heavy n) and compares the first sample[0] light / sample[1] heavy
    verdicts with the oracle's."""
    import torch
    from contact_props import check_contact_info
    dev = "cuda"
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    f = _f(fn)
    n_light, n_heavy = counts(n_ratio)
    res = []
    for heavy, total, ch, ns in ((False, n_light, chunk, sample[0]), (True, n_heavy, chunk_heavy, sample[1])):
        fails = 0
        for off in range(0, total, ch):
            n = min(ch, total - off)
            a, b = gen_a(n, g, dev), gen_b(n, g, dev)
            ok = ci.check(f, a, b, heavy, small_eps)
            fails += int((~ok).sum())
            if off == 0 and ns:
                of = _oracle_f(fn)
                got = ok[:ns].cpu().numpy()
                ar, br = a[:ns].cpu().numpy(), b[:ns].cpu().numpy()
                want = np.array([check_contact_info(of, ci.to_oracle(ar[k]), ci.to_oracle(br[k]), heavy=heavy,
                                                    small_eps=small_eps) for k in range(ns)])
                assert np.array_equal(got, want), np.argwhere(got != want)[:5]
        torch.cuda.synchronize()
        res += [fails, total]
    return res[0], res[2], res[1], res[3]


def test_circle_vs_circle_reference_scale(ci):
    # test/test_collisions.py:208-223: N = 10M, seed PRNGKey(1)
    fl, fh, nl, nh = _run(ci, 1, ci.rand_circles, ci.rand_circles, 1.0, 1e-5, seed=1, sample=(2000, 100))
    assert nl == 10_010_000 and nh == 200_200
    assert fl == 0 and fh == 0, (fl, fh)


def test_circle_vs_aabb_reference_scale(ci):
    # test/test_collisions.py:281-300: N_ratio 0.2, seed PRNGKey(0)
    fl, fh, nl, nh = _run(ci, 2, ci.rand_circles, ci.rand_aabbs, 0.2, 1e-5, seed=0, sample=(2000, 100))
    assert nl == 2_010_000 and nh == 40_200
    assert fl == 0 and fh == 0, (fl, fh)


def test_circle_vs_aabb_literal_cases_heavy(ci):
    # test/test_collisions.py:226-278, each checked with heavy=True (its default)
    import torch
    from test_oracle_geometry import CIRCLE_AABB_CASES
    n = len(CIRCLE_AABB_CASES)
    a = torch.zeros(n, 18, dtype=torch.float32)
    b = torch.zeros(n, 18, dtype=torch.float32)
    for k, (r, c, lo, up) in enumerate(CIRCLE_AABB_CASES):
        a[k, 2:5] = torch.tensor([r, c[0], c[1]])
        b[k, 0] = 1
        b[k, 2:6] = torch.tensor([lo[0], lo[1], up[0], up[1]])
    ok = ci.check(_f(2), a.cuda(), b.cuda(), True)
    assert bool(ok.all()), ok


SQUARE = [[0.5, 0.5], [-0.5, -0.5], [0.5, -0.5], [-0.5, 0.5]]
QUAD = [[0.3, 0.556], [-0.1, -0.2], [0.4, -0.3], [-0.8, 1.5]]
POLY_CASES = {
    # name: (contact fn, shape a, shape b, reference seed) -- test/test_collisions.py:403-462
    "aabb_vs_polygon_rand": (4, "aabb", SQUARE, 2),
    "aabb_vs_polygon_rand_2": (4, "aabb", QUAD, 3),
    "polygon_vs_polygon_rand": (3, 3, QUAD, 4),
    "polygon_vs_polygon_rand_2": (3, 6, QUAD, 5),
}


@pytest.mark.parametrize("name", sorted(POLY_CASES))
def test_polygon_invariants_reference_skips(ci, name):
    fn, sa, verts_b, seed = POLY_CASES[name]
    gen_a = ci.rand_aabbs if sa == "aabb" else (lambda n, g, dev: ci.rand_polys(n, sa, g, dev))

    def gen_b(n, g, dev):
        return ci.fixed_polys(n, verts_b, dev)
    fl, fh, nl, nh = _run(ci, fn, gen_a, gen_b, 0.1, 1e-3, seed=seed, chunk=1_010_000, chunk_heavy=20_200,
                          sample=(300, 40))
    assert nl == 1_010_000 and nh == 20_200
    line = "%s: light %d/%d pass (%.5f), heavy %d/%d pass (%.5f)" % (name, nl - fl, nl, 1 - fl / nl, nh - fh, nh,
                                                                       1 - fh / nh)
    print(line)
    out = os.environ.get("COTIX_INVARIANTS_LOG")
    if out:
        with open(out, "a") as fh_:
            fh_.write(line + "\n")
    if name == "polygon_vs_polygon_rand_2":
        # Polygon(jr.normal(k, (6, 2))): six random points sorted by angle are
        # mostly NOT convex, outside what GJK/EPA assume -- measured on MI355X:
        # 0.661 of the light and 0.662 of the heavy cases pass (profiles/r02f_invariants.txt)
        assert 0.6 < 1 - fl / nl < 0.72 and 0.6 < 1 - fh / nh < 0.72
    else:  # convex shapes: every case passes, as the reference asserts for its enabled tests
        assert fl == 0 and fh == 0, line
