"""Shared cases for the differentiable-rollout tests (CPU emulation and GPU).

box world: one scene (tests/golden/make_golden.box_world_bodies(0): three
static walls + four finite-mass balls), each env with its own random ball
states, so circle-circle, circle-AABB contacts and sustained resolutions are
exercised.  robocup: the bench batch (cotix/_robocup.py scene)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import make_golden as mg  # noqa: E402
from cotix_oracle import grad as G  # noqa: E402
from cotix_oracle import physics as P  # noqa: E402
from cotix_oracle import prng  # noqa: E402

D0 = prng.gjk_initial_direction()


def box_case(B, T, seed=0):
    make = lambda: mg.box_world_bodies(0)  # noqa: E731
    base = np.array([b.dyn() for b in make()], np.float32)
    rng = np.random.default_rng(seed)
    S0 = np.repeat(base[None], B, axis=0)
    for e in range(B):
        for b in range(3, 7):
            S0[e, b] = [rng.uniform(-2.5, 2.5), rng.uniform(-1.6, 1.6), rng.uniform(-3, 3), rng.uniform(-3, 3),
                        rng.uniform(-1, 1), rng.uniform(-5, 5)]
    keys = np.asarray(prng.split(prng.PRNGKey(11 + seed), B), np.uint32)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(7 * 6, np.float32)
    w[6 * 6 + 0] = 1.0   # ball 6: x
    w[5 * 6 + 3] = 0.5   # ball 5: vy
    return dict(make=make, S0=S0.astype(np.float32), keys=keys, actions=actions, w=w, ab=6, step=P.robocup_step,
                tol=ANALYTIC_TOL, name="box")


def robocup_case(B, T, seed=0):
    from cotix_oracle import cport
    dyn, keys = cport.robocup_batch(B)
    rng = np.random.default_rng(seed)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(5 * 6, np.float32)
    w[4 * 6 + 0] = 1.0   # return = sum_t ball x
    return dict(make=P.robocup_bodies, S0=np.ascontiguousarray(dyn.transpose(2, 0, 1)), keys=keys,
                actions=actions, w=w, ab=4, step=P.robocup_step, tol=ANALYTIC_TOL, name="robocup")


def lunar_case(B, T, seed=0, drop=-0.02):
    """LunarLander (cotix/_lunar_lander.py) started with its legs on the landing
    pad (y = -2 between x = -2 and 2): polygon x polygon contacts (GJK/EPA,
    contact_from_edges) and the four joints from the first step.  Per env a
    random lander/leg velocity and a small common offset."""
    make = lambda: P.lunar_lander_bodies(prng.PRNGKey(0))  # noqa: E731
    base = np.array([b.dyn() for b in make()], np.float32)
    rng = np.random.default_rng(seed)
    S0 = np.repeat(base[None], B, axis=0)
    for e in range(B):
        dx, dy = rng.uniform(-0.3, 0.3), -(5.0 + 1.2) + drop + rng.uniform(-0.05, 0.05)
        for b in range(3):
            S0[e, b, 0] += dx
            S0[e, b, 1] += dy
            S0[e, b, 2] = rng.uniform(-0.5, 0.5)
            S0[e, b, 3] = rng.uniform(-1.0, 0.2)
            S0[e, b, 5] = rng.uniform(-0.5, 0.5)
    keys = np.asarray(prng.split(prng.PRNGKey(21 + seed), B), np.uint32)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(4 * 6, np.float32)
    w[0] = 1.0          # lander x
    w[1] = 0.5          # lander y
    w[4] = 2.0          # lander angle
    w[2 * 6 + 3] = 0.25  # left leg vy
    return dict(make=make, S0=S0.astype(np.float32), keys=keys, actions=actions, w=w, ab=0,
                step=P.lunar_lander_step, tol=POLYGON_TOL, name="lunar")


def poly_box_bodies(octagons=False):
    """A static AABB floor and wall with two dynamic polygons (a Polygon4 box
    and a Polygon6 hexagon, or two 8-gons) resting on the floor against each
    other: aabb_vs_polygon and polygon_vs_polygon contacts of rotating bodies
    (8-gon pairs have 80 contact_from_edges terms: the backward's in-chain
    path)."""
    from cotix_oracle import geometry as Gm
    floor = P.Body([Gm.AABB((-5.0, -1.0), (5.0, 0.0))], mass=np.inf, inertia=np.inf, elasticity=0.3,
                   friction_coefficient=0.4)
    wall = P.Body([Gm.AABB((-1.2, 0.0), (-0.9, 2.0))], mass=np.inf, inertia=np.inf, elasticity=0.3,
                  friction_coefficient=0.4)
    sq = Gm.Polygon([(-0.3, -0.3), (0.3, -0.3), (0.3, 0.3), (-0.3, 0.3)], kind="Polygon4")
    hexv = [(0.35 * np.cos(k * np.pi / 3), 0.35 * np.sin(k * np.pi / 3)) for k in range(6)]
    hx = Gm.Polygon(hexv, kind="Polygon6")
    if octagons:
        sq = Gm.Polygon([(0.32 * np.cos(k * np.pi / 4 + 0.3), 0.32 * np.sin(k * np.pi / 4 + 0.3)) for k in range(8)],
                        kind="Polygon")
        hx = Gm.Polygon([(0.35 * np.cos(k * np.pi / 4), 0.35 * np.sin(k * np.pi / 4)) for k in range(8)],
                        kind="Polygon")
    box = P.Body([sq], mass=1.0, inertia=0.06, position=(-0.55, 0.28), angle=0.1, elasticity=0.5,
                 friction_coefficient=0.3)
    hexa = P.Body([hx], mass=1.5, inertia=0.09, position=(0.1, 0.32), angle=0.05, elasticity=0.5,
                  friction_coefficient=0.3)
    return [floor, wall, box, hexa]


def poly_box_case(B, T, seed=0, octagons=False):
    make = lambda: poly_box_bodies(octagons)  # noqa: E731
    base = np.array([b.dyn() for b in make()], np.float32)
    rng = np.random.default_rng(seed)
    S0 = np.repeat(base[None], B, axis=0)
    for e in range(B):
        for b in (2, 3):
            S0[e, b, 0] += rng.uniform(-0.03, 0.03)
            S0[e, b, 1] += rng.uniform(-0.03, 0.0)
            S0[e, b, 2:4] = rng.uniform(-0.5, 0.5, 2)
            S0[e, b, 4] += rng.uniform(-0.1, 0.1)
            S0[e, b, 5] = rng.uniform(-1.0, 1.0)
    keys = np.asarray(prng.split(prng.PRNGKey(31 + seed), B), np.uint32)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(4 * 6, np.float32)
    w[2 * 6 + 0] = 1.0   # box x
    w[3 * 6 + 1] = 0.5   # hexagon y
    w[3 * 6 + 4] = 1.0   # hexagon angle
    return dict(make=make, S0=S0.astype(np.float32), keys=keys, actions=actions, w=w, ab=2, step=P.robocup_step,
                tol=POLYGON_TOL, name="octagons" if octagons else "poly_box")


def ball_poly_bodies():
    """Two balls on polygon terrain: a static Polygon4 floor and a static
    tilted Polygon4 ramp, two dynamic circles resting on them and on each
    other -- circle x polygon contacts (GJK + EPA with the circle's
    direction-dependent support, cotix/_contacts.py:157-202) and a circle x
    circle contact."""
    from cotix_oracle import geometry as Gm
    floor = P.Body([Gm.Polygon([(-4.0, -1.0), (4.0, -1.0), (4.0, 0.0), (-4.0, 0.0)], kind="Polygon4")],
                   mass=np.inf, inertia=np.inf, elasticity=0.3, friction_coefficient=0.4)
    ramp = P.Body([Gm.Polygon([(1.0, 0.0), (3.0, 0.0), (3.0, 1.0), (1.0, 0.2)], kind="Polygon4")],
                  mass=np.inf, inertia=np.inf, elasticity=0.3, friction_coefficient=0.4)
    b1 = P.Body([Gm.Circle(0.3, (0.0, 0.0))], mass=1.0, inertia=0.05, position=(0.0, 0.29),
                elasticity=0.6, friction_coefficient=0.3)
    b2 = P.Body([Gm.Circle(0.25, (0.0, 0.0))], mass=0.7, inertia=0.03, position=(0.54, 0.24),
                elasticity=0.6, friction_coefficient=0.3)
    return [floor, ramp, b1, b2]


def ball_poly_case(B, T, seed=0):
    make = ball_poly_bodies
    base = np.array([b.dyn() for b in make()], np.float32)
    rng = np.random.default_rng(seed)
    S0 = np.repeat(base[None], B, axis=0)
    for e in range(B):
        for b in (2, 3):
            S0[e, b, 0] += rng.uniform(-0.02, 0.02)
            S0[e, b, 1] += rng.uniform(-0.02, 0.0)
            S0[e, b, 2:4] = rng.uniform(-0.4, 0.4, 2)
            S0[e, b, 5] = rng.uniform(-1.0, 1.0)
    keys = np.asarray(prng.split(prng.PRNGKey(51 + seed), B), np.uint32)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(4 * 6, np.float32)
    w[2 * 6 + 0] = 1.0   # ball 1 x
    w[3 * 6 + 1] = 0.5   # ball 2 y
    w[3 * 6 + 5] = 0.25  # ball 2 angular velocity
    return dict(make=make, S0=S0.astype(np.float32), keys=keys, actions=actions, w=w, ab=2, step=P.robocup_step,
                tol=POLYGON_TOL, name="ball_poly")


def quad_row_case(B, T, seed=0):
    """Nine Polygon4 bodies (one contact-type key): a static floor quad and a
    row of eight touching boxes on it -- 24 * nb words exceed the key window,
    so the backward does the GJK/EPA contact VJPs inside its serial chain."""
    from cotix_oracle import geometry as Gm

    def make():
        floor = P.Body([Gm.Polygon([(-6, -1), (6, -1), (6, 0), (-6, 0)], kind="Polygon4")], mass=np.inf,
                       inertia=np.inf, elasticity=0.2, friction_coefficient=0.5)
        out = [floor]
        for q in range(8):
            sq = Gm.Polygon([(-0.25, -0.25), (0.25, -0.25), (0.25, 0.25), (-0.25, 0.25)], kind="Polygon4")
            out.append(P.Body([sq], mass=1.0, inertia=0.04, position=(-2.0 + 0.49 * q, 0.24), angle=0.02 * q,
                              elasticity=0.4, friction_coefficient=0.3))
        return out
    base = np.array([b.dyn() for b in make()], np.float32)
    rng = np.random.default_rng(seed)
    S0 = np.repeat(base[None], B, axis=0)
    for e in range(B):
        for b in range(1, 9):
            S0[e, b, 2:4] = rng.uniform(-0.3, 0.3, 2)
            S0[e, b, 5] = rng.uniform(-0.5, 0.5)
    keys = np.asarray(prng.split(prng.PRNGKey(41 + seed), B), np.uint32)
    actions = (rng.normal(size=(T, B, 2)) * 0.1).astype(np.float32)
    w = np.zeros(9 * 6, np.float32)
    w[4 * 6 + 0] = 1.0
    w[5 * 6 + 4] = 0.5
    return dict(make=make, S0=S0.astype(np.float32), keys=keys, actions=actions, w=w, ab=4, step=P.robocup_step,
                tol=POLYGON_TOL, name="quad_row")


def oracle(case, envs=None, params=None):
    """Per env: (ret, grad_actions [T,2], grad_S0 [nb,6]) from the torch VJP
    chain, under the oracle parameter block `params` (None: the defaults)."""
    from cotix_oracle import params as _params
    B = case["S0"].shape[0]
    envs = range(B) if envs is None else envs
    out = {}
    with _params.use(params):
        d0 = prng.gjk_initial_direction()  # random_direction(PRNGKey(1)) in the block's PRNG layout
        for e in envs:
            ret, ga, gS, _ = G.rollout_grad(case["make"], case["S0"][e], case["keys"][e], case["actions"][:, e],
                                            case["w"], case["ab"], d0, step=case["step"])
            out[e] = (ret, ga, gS)
    return out


def _oracle_worker(job):
    import torch
    torch.set_num_threads(1)
    case, envs, params = job
    return oracle(case, envs, params)


def oracle_parallel(case, envs, params=None, workers=8):
    """oracle() over `envs` in `workers` spawned processes (CPU only: a fresh
    interpreter each, nothing inherited from a parent that holds a GPU
    context), for the full-size checks that sample many envs."""
    import multiprocessing as mp
    envs = list(envs)
    workers = max(1, min(workers, len(envs)))
    if workers == 1:
        return oracle(case, envs, params)
    chunks = [envs[i::workers] for i in range(workers)]
    out = {}
    with mp.get_context("spawn").Pool(workers) as pool:
        for part in pool.map(_oracle_worker, [(case, ch, params) for ch in chunks]):
            out.update(part)
    return out


# Gradient tolerances, measured: the kernel's
# hand-written f32 VJPs against the oracle's torch-f32 autograd of the same
# forward differ by rounding only, so the check is north_star's 1e-5
# relative, elementwise.  Scenes with GJK/EPA contacts add an absolute part,
# FLOOR * max|want| of the gradient block: their gradient entries are sums of
# large terms of both signs (contact_from_edges' terms, the polygon vertex
# chains), whose f32 rounding is relative to the terms, not to the small sum.
# Measured (tests/test_grad_cpu.py, host emulation == GPU bit for bit; the
# floor each case needs at rtol 1e-5): RoboCup 0 on the small cases, but
# 2.24e-7 at full size (config 5, 4096 x 64: env 2722's d/d action[0], -2.1900
# vs -2.1899 within a block whose max |want| is 175 -- the first step's
# gradient sums the whole 64-step chain; 1 of the 32 finite-gradient envs the
# full-size test samples); box world 0 at 40 steps and 5.75e-9 at 32 (one
# dyn0 entry near zero, the sum of the two walls' terms); LunarLander 1.3e-10;
# quad row 8.1e-8; polygon box 5.0e-7; octagon pair 1.19e-6 --
# ANALYTIC_TOL's 1e-6 is 4.5x RoboCup's full-size need, POLYGON_TOL's 4e-6
# 3.4x the largest.
ANALYTIC_TOL = (1e-5, 1e-6)
POLYGON_TOL = (1e-5, 4e-6)
MEASURED = {}  # name -> the floor the compared blocks needed at rtol 1e-5 (reported by conftest)


def close(got, want, tol=ANALYTIC_TOL, name=None):
    """Gradient agreement: the same NaN pattern, and for every entry
    |got - want| <= rtol |want| + floor max|want| (tol = (rtol, floor), the
    max over the finite entries of this block)."""
    rtol, floor = tol
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    ng, nw = np.isnan(got), np.isnan(want)
    if not np.array_equal(ng, nw):
        return False, "NaN pattern differs (%d vs %d)" % (ng.sum(), nw.sum())
    g, w = got[~nw], want[~nw]
    if g.size == 0:
        return True, ""
    mx = np.max(np.abs(w))
    d = np.abs(g - w)
    need = float(np.max(np.maximum(d - rtol * np.abs(w), 0.0)) / mx) if mx > 0 else float(np.max(d))
    if name is not None:
        MEASURED[name] = max(MEASURED.get(name, 0.0), need)
    ok = bool(np.all(d <= rtol * np.abs(w) + floor * mx))
    rel = float(np.max(d / np.maximum(np.abs(w), 1e-300)))
    return ok, "needs floor %.3g at rtol %g (allowed %g); max relative error %.3g" % (need, rtol, floor, rel)
