"""TEST INFRASTRUCTURE ONLY -- CPU oracle, never imported by the product path.

Scalar float32 restatement of cotix's dynamics and scenarios:
  cotix/_bodies.py               AnyBody / DynamicBody state, velocity_at, load
  cotix/_physics_solvers.py      ExplicitEulerPhysics
  cotix/_collision_resolution.py resolve_collision / apply_impulse
  cotix/_colliders.py            RandomizedCollider.resolve
  cotix/_constraint_solvers.py   SimpleConstraintSolver (identity: no constraint
                                 class exists in the reference)
  cotix/_robocup.py              RoboCupEnv.__init__
  cotix/_lunar_lander.py         LunarLander.__init__ / .step
  examples/test_viz.py:24-44,61-69  the step composition

The collider is restated *faithfully*: the full N1 x N2 cross product of
candidates, evaluated in the reference's scan order (ind2 outer, ind1 inner),
one bernoulli per candidate, "last write wins".  The only deliberate deviation
is the candidate order: the reference passes the candidate lists through
``list(set(...))`` of id-hashed tracers (cotix/_colliders.py:116-120), which
is not reproducible run to run; the build uses insertion order.
"""
import copy

import numpy as np

from . import params as _params
from . import prng
from .geometry import (AABB, CONTACT_FUNCS, clip, F, NAN, NAN_CONTACT, ONE, ZERO, Circle, ErrorFlag,
                       Polygon, Transformer, contact_isnan, cross, dot, fmin, norm, run_contact,
                       sincos32, vadd, vneg, vscale, vsub)

INF = F(np.inf)


class Body:
    """AnyBody (cotix/_bodies.py:135-186): dynamic state + static parameters +
    a list of convex parts in local coordinates (UniversalShape.parts)."""

    def __init__(self, parts, mass=1.0, inertia=1.0, position=(0.0, 0.0), velocity=(0.0, 0.0),
                 angle=0.0, angular_velocity=0.0, elasticity=1.0, friction_coefficient=1.0,
                 is_area=False):
        self.parts = list(parts)
        self.mass = F(mass)
        self.inertia = F(inertia)
        self.position = (F(position[0]), F(position[1]))
        self.velocity = (F(velocity[0]), F(velocity[1]))
        self.angle = F(angle)
        self.angular_velocity = F(angular_velocity)
        self.elasticity = F(elasticity)
        self.friction_coefficient = F(friction_coefficient)
        self.is_area = is_area

    def transformer(self):
        """shape._transformer after update_transform (cotix/_bodies.py:37-48)."""
        return Transformer(self.position, self.angle)

    def velocity_at(self, point):  # cotix/_bodies.py:50-55
        r = vsub(point, self.position)
        perp = (-r[1], r[0])
        return (self.velocity[0] + perp[0] * self.angular_velocity,
                self.velocity[1] + perp[1] * self.angular_velocity)

    def dyn(self):
        return [self.position[0], self.position[1], self.velocity[0], self.velocity[1],
                self.angle, self.angular_velocity]

    def set_dyn(self, d):
        self.position = (F(d[0]), F(d[1]))
        self.velocity = (F(d[2]), F(d[3]))
        self.angle = F(d[4])
        self.angular_velocity = F(d[5])


def clone_bodies(bodies):
    return [copy.copy(b) for b in bodies]


# ----------------------------------------------------------------------------
# ExplicitEulerPhysics (cotix/_physics_solvers.py:16-33)
# ----------------------------------------------------------------------------
def euler_step(bodies, dt):
    dt = F(dt)
    for b in bodies:
        b.position = (b.position[0] + b.velocity[0] * dt, b.position[1] + b.velocity[1] * dt)
        b.angle = b.angle + b.angular_velocity * dt
    return bodies


# ----------------------------------------------------------------------------
# resolve_collision (cotix/_collision_resolution.py:52-151)
# ----------------------------------------------------------------------------
def apply_impulse(body, impulse, point):  # :68-73
    arm = vsub(point, body.position)
    torque = cross(arm, impulse)
    body.velocity = (body.velocity[0] + impulse[0] / body.mass,
                     body.velocity[1] + impulse[1] / body.mass)
    body.angular_velocity = body.angular_velocity + torque / body.inertia


def resolve_collision(b1, b2, contact):
    pen, cp = contact
    if contact_isnan(contact):  # :52-65
        return
    v1 = b1.velocity_at(cp)
    v2 = b2.velocity_at(cp)
    relv = vsub(v2, v1)
    pn = norm(pen)
    n = (pen[0] / pn, pen[1] / pn)
    vn = dot(relv, n)
    e = fmin(b1.elasticity, b2.elasticity)
    r1 = vsub(cp, b1.position)
    r2 = vsub(cp, b2.position)
    lever1 = r1[0] * r1[0] + r1[1] * r1[1]
    lever2 = r2[0] * r2[0] + r2[1] * r2[1]
    ang = lever1 / b1.inertia + lever2 / b2.inertia
    prm = _params.current()  # baumgarte_term 0.3 (:105) and the divisor 0.01 (:115)
    nim = (-(ONE + e)) * vn - (F(prm.baumgarte) * norm(pen)) / F(prm.baumgarte_dt)
    den = (ONE / b1.mass + ONE / b2.mass) + ang
    ni = nim / den
    imp = vscale(n, ni)
    mu = (b1.friction_coefficient + b2.friction_coefficient) / F(2)
    vd = (relv[0] + vn * n[0], relv[1] + vn * n[1])
    vdn = norm(vd)
    vdu = (vd[0] / vdn, vd[1] / vdn)
    idr = (-vdn) / ((ONE / b1.mass + ONE / b2.mass) + ang)
    idr = clip(idr, ZERO, ni * mu)
    imp = vadd(imp, vscale(vdu, idr))
    if dot(pen, relv) < 0:  # :139-148: moving apart -> nothing
        return
    apply_impulse(b1, vneg(imp), cp)
    apply_impulse(b2, imp, cp)


# ----------------------------------------------------------------------------
# RandomizedCollider (cotix/_colliders.py:74-351)
# ----------------------------------------------------------------------------
def enumerate_candidates(bodies):
    """Trace-time enumeration (:86-113): dict insertion order of type keys;
    per key two lists of (body index, part index).  Canonical order =
    insertion order (the reference's set() permutation is not reproducible)."""
    type_to = {}
    for i, body in enumerate(bodies):
        for j, body2 in enumerate(bodies):
            if i <= j:
                continue
            for pa, a in enumerate(body.parts):
                for pb, b in enumerate(body2.parts):
                    t1, t2 = a.kind, b.kind
                    if (t1, t2) in CONTACT_FUNCS:
                        pass
                    elif (t2, t1) in CONTACT_FUNCS:
                        t1, t2 = t2, t1
                    else:
                        raise RuntimeError("illegal shape pair %s/%s" % (t1, t2))
                    l1, l2 = type_to.setdefault((t1, t2), ([], []))
                    l1.append((i, pa))
                    l2.append((j, pb))
    return type_to


def collider_resolve(bodies, rkey, d0, err=None, trace=None):
    """RandomizedCollider.resolve, faithful restatement (forward scan)."""
    n = len(bodies)
    type_to = enumerate_candidates(bodies)
    tfs = [b.transformer() for b in bodies]
    world = [[p.transform(tfs[bi]) for p in b.parts] for bi, b in enumerate(bodies)]

    pen = [[(ZERO, ZERO) for _ in range(n)] for _ in range(n)]
    cp = [[(NAN, NAN) for _ in range(n)] for _ in range(n)]
    src = [[None for _ in range(n)] for _ in range(n)]  # (contact fn, (body, part) of s1, of s2)
    win = [[-1 for _ in range(n)] for _ in range(n)]  # winning candidate: ind1 | ind2 << 9 | type << 18
    skey = prng.split(rkey)[0]  # :142
    for ti, (key_t, (l1, l2)) in enumerate(type_to.items()):
        N1, N2 = len(l1), len(l2)
        fname = CONTACT_FUNCS[key_t]
        # cross product of contacts :149-173
        cur = [[None] * N2 for _ in range(N1)]
        srcs = {}
        for i1, (bi, pi) in enumerate(l1):
            for i2, (bj, pj) in enumerate(l2):
                s1 = world[bi][pi]
                s2 = world[bj][pj]
                o1, o2 = (bi, pi), (bj, pj)
                if (s1.kind, s2.kind) not in CONTACT_FUNCS:  # :155-157
                    s1, s2 = s2, s1
                    o1, o2 = o2, o1
                srcs[(i1, i2)] = (fname, o1, o2)
                # the contact is evaluated for every pair (so error_if trips
                # count for i < j too) and then masked by lax.cond(i < j) :163
                c = run_contact(fname, s1, s2, d0, err)
                cur[i1][i2] = NAN_CONTACT if bi < bj else c
        skey = prng.split(skey)[0]  # :175
        keys2 = prng.split(skey, N2)
        for i2 in range(N2):  # scan over ind2 (outer) :259-267
            keys1 = prng.split(keys2[i2], N1)
            for i1 in range(N1):  # scan over ind1 (inner) :249-256
                c = cur[i1][i2]
                if contact_isnan(c):
                    continue  # bernoulli draw has no effect on a NaN candidate
                k1 = prng.split(keys1[i1])[0]  # :222
                if prng.bernoulli(k1, _params.current().contact_p):  # :220-223, :235-239
                    bi, bj = l1[i1][0], l2[i2][0]
                    pen[bi][bj] = c[0]
                    cp[bi][bj] = c[1]
                    src[bi][bj] = srcs[(i1, i2)]
                    win[bi][bj] = i1 | (i2 << 9) | (ti << 18)
    # choose_random_contact :274-295
    ckeys = prng.split(skey, n)
    chosen = []
    for i in range(n):
        good = [not (np.isnan(cp[i][j][0]) or np.isnan(cp[i][j][1])) for j in range(n)]
        cnt = sum(good)
        if cnt == 0:
            chosen.append(i)
            continue
        p = [F(1.0 if g else 0.0) / F(cnt) for g in good]
        chosen.append(prng.choice_p(ckeys[i], n, p))
    if trace is not None:
        trace["chosen"] = list(chosen)
        trace["contacts"] = [[(pen[i][j], cp[i][j]) for j in range(n)] for i in range(n)]
        trace["src"] = src
        trace["cells"] = [row[:] for row in win]
    # sequential resolution :310-336
    for i in range(n):
        j = chosen[i]
        if i == j:
            continue
        resolve_collision(bodies[i], bodies[j], (pen[i][j], cp[i][j]))
    return bodies


# ----------------------------------------------------------------------------
# scenarios
# ----------------------------------------------------------------------------
def robocup_bodies():
    """RoboCupEnv.__init__ (cotix/_robocup.py:14-130), every constant in f32
    exactly as the JAX expressions produce it."""
    field_dim = (F(10.4), F(7.4))
    f2 = F(2)
    field = AABB((-field_dim[0] / f2, -field_dim[1] / f2), (field_dim[0] / f2, field_dim[1] / f2))
    # play_area_dim=(9, 6) is an int32 array; /2 -> f32
    play = AABB((F(-9) / f2, F(-6) / f2), (F(9) / f2, F(6) / f2))
    gd0, gd1 = F(0.2), F(1.0)
    yb_lo = (play.lower[0] - gd0, F(-1.0 / 2))
    yb_up = (play.lower[0], F(1.0 / 2))
    gw = F(0.01)
    ya = AABB(yb_lo, (yb_lo[0] + gw, yb_lo[1] + gd1))
    yb = AABB((yb_lo[0] - (-gw), yb_lo[1] - ZERO), (yb_lo[0] + gd0, yb_lo[1] + gw))
    yc = AABB((yb_up[0] - gd0, yb_up[1] - gw), yb_up)

    def refl(a):
        return AABB((-a.upper[0], a.lower[1]), (-a.lower[0], a.upper[1]))

    ball_r = F(0.022) * F(3)
    field_body = Body([field], mass=INF, is_area=True)
    play_body = Body([play], mass=INF, is_area=True)
    yellow = Body([ya, yb, yc], mass=INF, elasticity=0.5)
    blue = Body([refl(ya), refl(yb), refl(yc)], mass=INF, elasticity=0.5)
    ball = Body([Circle(ball_r, (0.0, 0.0))], mass=0.5, velocity=(1.0, 0.01),
                angular_velocity=10.0, elasticity=1.0)
    return [field_body, play_body, yellow, blue, ball]


LANDER_POLY = [(-14, 17), (-17, 0), (-17, -10), (17, -10), (17, 0), (14, 17)]
LEG_AWAY, LEG_DOWN, LEG_W, LEG_H, LEG_ANGLE = 24, 8, 2, 8, -0.3


def lunar_lander_bodies(key=None):
    """LunarLander.__init__ (cotix/_lunar_lander.py:29-143)."""
    if key is None:
        key = prng.PRNGKey(0)
    f05 = F(0.05)
    lander_shape = Polygon([(F(x) * f05, F(y) * f05) for x, y in LANDER_POLY], kind="Polygon6")
    # legs: int vertices sorted, then rotated (v @ R) and scaled WITHOUT
    # re-sorting (eqx.tree_at bypasses __init__), right leg mirrored.
    leg = Polygon([(-LEG_W, -LEG_H), (LEG_W, -LEG_H), (LEG_W, LEG_H), (-LEG_W, LEG_H)], kind="Polygon4")
    s, c = sincos32(F(LEG_ANGLE))
    rot = [(v[0] * c + v[1] * s, v[0] * (-s) + v[1] * c) for v in leg.vertices_]
    lverts = [(v[0] * f05, v[1] * f05) for v in rot]
    rverts = [(v[0] * F(-1.0), v[1] * F(1.0)) for v in lverts]
    left_leg_shape = Polygon(lverts, kind="Polygon4", sort=False)
    right_leg_shape = Polygon(rverts, kind="Polygon4", sort=False)
    center = (ZERO, F(5.0))
    lleg_pos = (F(LEG_AWAY) * f05 + center[0], F(-LEG_DOWN) * f05 + center[1])
    rleg_pos = (F(-LEG_AWAY) * f05 + center[0], F(-LEG_DOWN) * f05 + center[1])
    lander = Body([lander_shape], mass=30.0, inertia=30.0, position=center, angle=0.01,
                  friction_coefficient=0.1)
    right_leg = Body([right_leg_shape], inertia=1.0, position=rleg_pos, friction_coefficient=0.1)
    left_leg = Body([left_leg_shape], inertia=1.0, position=lleg_pos, friction_coefficient=0.1)
    ground_polys = lunar_lander_terrain(key)
    ground = Body([Polygon(p, kind="Polygon4") for p in ground_polys], mass=INF, inertia=INF,
                  elasticity=0.1, friction_coefficient=0.1)
    return [lander, right_leg, left_leg, ground]


def lunar_lander_terrain(key):
    """cotix/_lunar_lander.py:109-132: 7 unsorted quads (sorted by Polygon4)."""
    k1, k2, k3, k4, k5 = prng.split(key, 5)
    h = list(prng.uniform(k1, (8,), -5.0, 5.0))
    h[0] = h[0] * F(10)
    h[3] = F(-2.0)
    h[-4] = F(-2.0)
    h[-1] = h[-1] * F(10)
    pos = [F(-100), prng.uniform(k2, (), -12.0, -9.0)[()], prng.uniform(k3, (), -8.0, -4.0)[()],
           F(-2), F(2), prng.uniform(k4, (), 4.0, 8.0)[()], prng.uniform(k5, (), 9.0, 12.0)[()], F(100)]
    polys = []
    for i in range(7):
        polys.append([(pos[i], h[i]), (pos[i], F(-10)), (pos[i + 1], h[i + 1]), (pos[i + 1], F(-10))])
    return polys


def lunar_lander_constraints(bodies):
    """LunarLander.step (cotix/_lunar_lander.py:145-218)."""
    from .geometry import rotate
    f05 = F(0.05)
    lander, right_leg, left_leg = bodies[0], bodies[1], bodies[2]
    llj1 = vadd(rotate((F(LEG_AWAY) * f05, F(-LEG_DOWN) * f05), lander.angle), lander.position)
    llj2 = vadd(rotate((F(LEG_AWAY) * f05, F(-LEG_DOWN + 8) * f05), lander.angle), lander.position)
    lj1 = left_leg.position
    lj2 = vadd(left_leg.position, rotate((ZERO, F(0.4)), left_leg.angle))
    lrj1 = vadd(rotate((F(-LEG_AWAY) * f05, F(-LEG_DOWN) * f05), lander.angle), lander.position)
    lrj2 = vadd(rotate((F(-LEG_AWAY) * f05, F(-LEG_DOWN + 8) * f05), lander.angle), lander.position)
    rj1 = right_leg.position
    rj2 = vadd(right_leg.position, rotate((ZERO, F(0.4)), right_leg.angle))

    def fixed(b1, c1, b2, c2):
        dp = vsub(c1, c2)
        dv = vsub(b1.velocity_at(c1), b2.velocity_at(c2))
        k = norm(dv) + F(0.1)
        imp = (dp[0] * ONE + (dv[0] * k) * f05, dp[1] * ONE + (dv[1] * k) * f05)
        apply_impulse(b1, vneg(imp), c1)
        apply_impulse(b2, imp, c2)

    fixed(lander, llj1, left_leg, lj1)
    fixed(lander, llj2, left_leg, lj2)
    fixed(lander, lrj1, right_leg, rj1)
    fixed(lander, lrj2, right_leg, rj2)
    right_leg.angular_velocity = right_leg.angular_velocity * F(0.95)
    left_leg.angular_velocity = left_leg.angular_velocity * F(0.95)
    return bodies


# ----------------------------------------------------------------------------
# step drivers (examples/test_viz.py)
# ----------------------------------------------------------------------------
DT = 1e-2
LL_GRAVITY = -0.002


def apply_action(bodies, action, action_body):
    """Config-5 action: velocity += action after Euler."""
    if action is None:
        return
    v = bodies[action_body].velocity
    bodies[action_body].velocity = (v[0] + F(action[0]), v[1] + F(action[1]))


def robocup_step(bodies, key, d0, err=None, trace=None, dt=DT, action=None, action_body=None):
    """examples/test_viz.py:61-69: Euler -> collider -> (identity constraint
    pass) -> key = split(key)[0]."""
    euler_step(bodies, dt)
    apply_action(bodies, action, action_body)
    collider_resolve(bodies, key, d0, err, trace)
    return bodies, prng.split(key)[0]


def lunar_lander_step(bodies, key, d0, err=None, trace=None, dt=DT, action=None, action_body=None):
    """examples/test_viz.py:24-44."""
    euler_step(bodies, dt)
    v = bodies[0].velocity
    bodies[0].velocity = (v[0] + ZERO, v[1] + F(LL_GRAVITY))
    apply_action(bodies, action, action_body)
    collider_resolve(bodies, key, d0, err, trace)
    nxt = prng.split(key)[0]
    lunar_lander_constraints(bodies)
    return bodies, nxt
