"""Pins the oracle's geometry/narrowphase restatement against every literal
and property the reference's own tests hold for this path:
test/test_shapes.py, test/test_collisions.py, test/test_physics_solvers.py,
test/test_geometry_utils.py."""
import numpy as np
import pytest

from contact_props import check_contact_info
from cotix_oracle import geometry as G
from cotix_oracle import physics as P

F = np.float32

# test/test_collisions.py:229-272 (circle radius, position; AABB lower, upper)
CIRCLE_AABB_CASES = [
    (4.808976, (0.52343243, 0.38244677), (1.2948408, 1.4734308), (3.3397233, 6.3817973)),
    (1.0, (1.0, 1.0), (-2.0, -2.0), (0.4, 0.7)),
    (5.0, (0.0, 0.0), (-2.0, -2.0), (2.0, 2.0)),
    (3.7427633, (-0.0277214, 1.0449156), (-0.6238362, -1.1297362), (1.3405488, -0.5544366)),
    (0.5361439, (-0.4457733, 0.5882554), (-0.44587463, -0.73396504), (0.0717122, 3.0028129)),
    (1.0, (0.0, 0.0), (-2.0, -2.0), (2.0, 2.0)),
    (0.01, (0.0, 1.8), (-2.0, -2.0), (2.0, 2.0)),
    (1.0, (0.1, 0.2), (-2.0, -2.3), (2.0, 2.0)),
    (1.0, (-0.3, 0.05), (-2.1, -2.3), (2.0, 2.0)),
    (1.0, (-0.12, -0.56), (-2.0, -2.0), (2.2, 2.3)),
]


@pytest.mark.parametrize("case", CIRCLE_AABB_CASES)
def test_circle_vs_aabb_parametrized(case):
    r, c, lo, up = case
    assert check_contact_info(G.circle_vs_aabb, G.Circle(r, c), G.AABB(lo, up), heavy=True)


def _rand_circle(rng):
    return G.Circle(F(rng.uniform(0.01, 5.0)), (F(rng.normal()), F(rng.normal())))


def _rand_aabb(rng):
    lo = np.array([rng.normal(), rng.normal()], F)
    up = lo + np.array([rng.uniform(0.01, 5.0), rng.uniform(0.01, 5.0)], F)
    return G.AABB(tuple(lo), tuple(up))


def test_circle_vs_circle_rand():
    # test/test_collisions.py:208-223 (10M cases there; a seeded sample here)
    rng = np.random.default_rng(1)
    for k in range(300):
        assert check_contact_info(G.circle_vs_circle, _rand_circle(rng), _rand_circle(rng), heavy=k % 10 == 0)


def test_circle_vs_aabb_rand():
    # test/test_collisions.py:281-300
    rng = np.random.default_rng(0)
    for k in range(300):
        assert check_contact_info(G.circle_vs_aabb, _rand_circle(rng), _rand_aabb(rng), heavy=k % 10 == 0)


def _global_support(parts, d):
    """UniversalShape.get_global_support (cotix/_universal_shape.py:44-58)
    with the identity transformer."""
    T = G.Transformer((0.0, 0.0), 0.0)
    sups = [T.forward_vector(p.support(d)) for p in parts]
    return sups[G.argmax([G.dot(s, d) for s in sups])]


def test_universal_shape_support_equivalence():
    # test/test_shapes.py:8-16
    c = G.Circle(0.1, (0.1, 0.2))
    rng = np.random.default_rng(42)
    for _ in range(100):
        d = (F(rng.normal()), F(rng.normal()))
        assert _global_support([c], d) == c.support(d)


def test_universal_shape_double_support_correctness():
    # test/test_shapes.py:19-35 (exact golden values)
    parts = [G.Circle(0.5, (-10.0, 0.0)), G.Circle(1.0, (1.0, 1.0))]
    assert _global_support(parts, (F(1), F(0))) == (2.0, 1.0)
    assert _global_support(parts, (F(-1), F(0))) == (-10.5, 0.0)
    assert _global_support(parts, (F(0), F(1))) == (1.0, 2.0)
    assert _global_support(parts, (F(0), F(-1))) == (-10.0, -0.5)


def test_simple_world_euler():
    # test/test_physics_solvers.py:9-40
    b = P.Body([G.Circle(1.0, (0.0, 0.0))], position=(0.1, 0.1), velocity=(1.0, 0.0))
    for _ in range(100):
        P.euler_step([b], 1e-1)
    assert b.position[0] > 2e-1
    assert 1e-1 - 1e-2 < b.position[1] < 1e-1 + 1e-2
    assert abs(b.parts[0].position[0]) < 1e-2 and abs(b.parts[0].position[1]) < 1e-2
    assert abs(b.velocity[0] - 1.0) < 1e-2


def test_order_clockwise_consistency():
    # test/test_geometry_utils.py:7-21
    rng = np.random.default_rng(42)
    verts = [tuple(v) for v in rng.uniform(size=(100, 2)).astype(F)]
    ref = G.order_clockwise(verts)
    for _ in range(100):
        perm = rng.permutation(100)
        assert G.order_clockwise([verts[k] for k in perm]) == ref


def test_sincos_atan2_accuracy():
    xs = np.linspace(-50, 50, 2001).astype(F)
    for x in xs:
        s, c = G.sincos32(x)
        assert abs(float(s) - np.sin(np.float64(x))) < 4e-7
        assert abs(float(c) - np.cos(np.float64(x))) < 4e-7
    rng = np.random.default_rng(3)
    for _ in range(2000):
        y, x = (F(v) for v in rng.normal(size=2) * 10)
        assert abs(float(G.atan2_32(y, x)) - np.arctan2(np.float64(y), np.float64(x))) < 6e-7
    for y, x in [(0.0, 1.0), (-0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0)]:
        assert float(G.atan2_32(F(y), F(x))) == pytest.approx(np.arctan2(y, x), abs=1e-7)
        assert np.signbit(G.atan2_32(F(y), F(x))) == np.signbit(np.arctan2(y, x))


def _rand_poly(rng, n, scale=1.0, center=(0.0, 0.0)):
    ang = np.sort(rng.uniform(0, 2 * np.pi, n))
    rad = rng.uniform(0.5, 1.0, n) * scale
    pts = [(F(center[0] + r * np.cos(a)), F(center[1] + r * np.sin(a))) for a, r in zip(ang, rad)]
    return G.Polygon(pts, kind="Polygon%d" % n)


def test_polygon_contacts_resolve_penetration(d0):
    """GJK+EPA: moving A by the penetration vector separates the shapes (the
    reference's skipped polygon tests assert the same invariant with a 1e-3
    tolerance, test/test_collisions.py:437-462)."""
    rng = np.random.default_rng(7)
    hits = 0
    for _ in range(150):
        a = _rand_poly(rng, 4, 1.0, tuple(rng.normal(size=2) * 0.6))
        b = _rand_poly(rng, 6, 1.0, (0.0, 0.0))
        pen, cp = G.polygon_vs_polygon(a, b, d0)
        if np.isnan(cp[0]):
            continue
        hits += 1
        pen2, cp2 = G.polygon_vs_polygon(a.move(pen), b, d0)
        assert np.isnan(cp2[0]) or G.norm(pen2) < 2e-3
    assert hits > 50
