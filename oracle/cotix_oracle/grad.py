"""TEST INFRASTRUCTURE ONLY -- the checker of the differentiable rollout
(BASELINE config 5).  Never imported by the product.

jax.grad of the reference step differentiates the executed branch of every
jax.lax.cond (cotix/_contacts.py:30-154, cotix/_collision_resolution.py:
52-146, cotix/_colliders.py:333) with argmin/argmax and the RandomizedCollider
choices as constants, and lax.max/min (jnp.clip) splitting ties 1/2-1/2.
This module restates the continuous part of one step with torch float32
autograd (torch.maximum/minimum have the same balanced tie rule), in the
oracle's exact operation order, so its forward values are bit-identical to
the oracle's and every branch/tie decision is the one the oracle took.  The
discrete choices (which contact each body resolves, and which part pair
produced it) come from the faithful oracle's trace (physics.collider_resolve
trace["src"]).  Gradients of a T-step return are chained step by step:
lambda_T = w; (lambda_t, dR/da_t) = VJP_t(lambda_{t+1}); lambda_t += w (t>=1).

Return definition: action a_t (f32[2]) is added
to the velocity of body `action_body` right after Euler; the return is
R = sum_{t=1..T} sum_k w_k * state_t[k] over terms with w_k != 0.
"""
import warnings

import numpy as np
import torch

from . import geometry as G
from . import params as _params
from . import physics as P

F32 = torch.float32
# branch decisions read forward values of graph tensors (intended)
warnings.filterwarnings("ignore", message="Converting a tensor with requires_grad=True to a scalar")


def _t(x):
    return torch.tensor(float(x), dtype=F32)


def _fmax(a, b):
    return torch.maximum(a, b)


def _fmin(a, b):
    return torch.minimum(a, b)


def _clip(x, lo, hi):  # jnp.clip = minimum(maximum(x, lo), hi)
    return _fmin(hi, _fmax(lo, x))


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1]


class _Sqrt(torch.autograd.Function):
    """Correctly rounded f32 sqrt (torch's CPU sqrt is not: it differs from
    IEEE sqrt in ~0.5% of f32 inputs, machine-dependently); JAX's JVP
    rule g * (0.5 / ans)."""

    @staticmethod
    def forward(ctx, x):
        y = torch.tensor(np.sqrt(np.float32(x.item())), dtype=F32)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return g * (0.5 / y)


def _norm(a):
    return _Sqrt.apply(a[0] * a[0] + a[1] * a[1])


def _cross(a, b):
    return a[0] * b[1] - a[1] * b[0]


def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def _add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def _isnan(v):
    return bool(torch.isnan(v[0])) or bool(torch.isnan(v[1]))


# ---- analytic contacts, contact branch (geometry.py / cotix/_contacts.py) ----
def circle_vs_circle(a, b):  # a, b = (radius, (cx, cy))
    ar, ap = a
    br, bp = b
    delta = _sub(ap, bp)
    distance = _norm(delta)
    if float(distance.detach()) == 0.0:
        direction = (_t(1.0), _t(0.0))
    else:
        direction = (delta[0] / distance, delta[1] / distance)
    m = _fmin(distance - (ar + br), _t(0.0))
    pen = (direction[0] * m, direction[1] * m)
    cp = ((bp[0] + direction[0] * (br - ar)) + ap[0], (bp[1] + direction[1] * (br - ar)) + ap[1])
    cp = (cp[0] / 2.0, cp[1] / 2.0)
    if not float(_dot(_sub(ap, cp), _sub(bp, cp))) <= 0:
        d = _sub(bp, ap)  # Circle.contains (geometry.py): sumsq(p - c) <= r*r, r = radius + eps
        r = np.float32(ar.item()) + np.float32(1e-6)
        inside = float(d[0] * d[0] + d[1] * d[1]) <= float(r * r)
        cp = bp if inside else ap
    assert float(distance) <= float(ar + br), "not a contact"
    return ((-pen[0], -pen[1]), cp)


def aabb_vs_aabb(a, b, eps=1e-8):  # a, b = (lower, upper)
    alo, aup = a
    blo, bup = b
    me = _t(-np.float32(eps))
    depths = [_fmax(aup[1] - blo[1], me), _fmax(bup[1] - alo[1], me), _fmax(aup[0] - blo[0], me),
              _fmax(bup[0] - alo[0], me)]
    dirs = [(0, -1), (0, 1), (-1, 0), (1, 0)]
    k = int(np.argmin([float(d) for d in depths]))
    md = _fmax(_t(0.0), depths[k])
    pen = (md * float(dirs[k][0]), md * float(dirs[k][1]))
    mu = (_fmin(aup[0], bup[0]), _fmin(aup[1], bup[1]))
    ml = (_fmax(alo[0], blo[0]), _fmax(alo[1], blo[1]))
    return (pen, ((mu[0] + ml[0]) / 2.0, (mu[1] + ml[1]) / 2.0))


def circle_vs_aabb(a, b, eps=1e-6):
    r, ap = a
    lo, up = b
    bc = ((lo[0] + up[0]) / 2.0, (lo[1] + up[1]) / 2.0)
    disp = _sub(ap, bc)
    l = _sub(lo, bc)
    h = _sub(up, bc)
    ccp = _add(bc, (_clip(disp[0], l[0], h[0]), _clip(disp[1], l[1], h[1])))
    vs = [lo, (lo[0], up[1]), up, (up[0], lo[1])]
    perfect = any(float(_norm(_sub(v, ccp)).detach()) < np.float32(eps) for v in vs)
    if perfect:
        d = _sub(ccp, ap)
        nd = _norm(d)
        dn = (d[0] / nd, d[1] / nd)
        q = _sub(_add(ap, (dn[0] * r, dn[1] * r)), ccp)
        return ((-q[0], -q[1]), ccp)
    shifts = [(ap[1] + r) - lo[1], up[1] - (ap[1] - r), (ap[0] + r) - lo[0], up[0] - (ap[0] - r)]
    dirs = [(0, 1), (0, -1), (1, 0), (-1, 0)]
    k = int(np.argmin([float(s) for s in shifts]))
    ns = -shifts[k]
    return ((ns * float(dirs[k][0]), ns * float(dirs[k][1])), ccp)


CONTACTS = {"circle_vs_circle": circle_vs_circle, "aabb_vs_aabb": aabb_vs_aabb, "circle_vs_aabb": circle_vs_aabb}


# ---- resolution (cotix/_collision_resolution.py:52-146) ----
class _B:
    def __init__(self, p, v, ang, w, body):
        self.p, self.v, self.ang, self.w = p, v, ang, w
        self.m, self.I = _t(body.mass), _t(body.inertia)
        self.e, self.mu = _t(body.elasticity), _t(body.friction_coefficient)

    def vel_at(self, pt):
        r = _sub(pt, self.p)
        return (self.v[0] + (-r[1]) * self.w, self.v[1] + r[0] * self.w)


def _apply(b, imp, pt):
    arm = _sub(pt, b.p)
    torque = _cross(arm, imp)
    b.v = (b.v[0] + imp[0] / b.m, b.v[1] + imp[1] / b.m)
    b.w = b.w + torque / b.I


def resolve(b1, b2, pen, cp):
    v1, v2 = b1.vel_at(cp), b2.vel_at(cp)
    relv = _sub(v2, v1)
    pn = _norm(pen)
    n = (pen[0] / pn, pen[1] / pn)
    vn = _dot(relv, n)
    e = _fmin(b1.e, b2.e)
    r1, r2 = _sub(cp, b1.p), _sub(cp, b2.p)
    lever1 = r1[0] * r1[0] + r1[1] * r1[1]
    lever2 = r2[0] * r2[0] + r2[1] * r2[1]
    ang = lever1 / b1.I + lever2 / b2.I
    prm = _params.current()  # cotix/_collision_resolution.py:105,115
    nim = (-(1.0 + e)) * vn - (_t(prm.baumgarte) * _norm(pen)) / _t(prm.baumgarte_dt)
    den = (1.0 / b1.m + 1.0 / b2.m) + ang
    ni = nim / den
    imp = (n[0] * ni, n[1] * ni)
    mu = (b1.mu + b2.mu) / 2.0
    vd = (relv[0] + vn * n[0], relv[1] + vn * n[1])
    vdn = _norm(vd)
    vdu = (vd[0] / vdn, vd[1] / vdn)
    idr = (-vdn) / ((1.0 / b1.m + 1.0 / b2.m) + ang)
    idr = _clip(idr, _t(0.0), ni * mu)
    imp = (imp[0] + vdu[0] * idr, imp[1] + vdu[1] * idr)
    if float(_dot(pen, relv)) < 0:
        return False
    _apply(b1, (-imp[0], -imp[1]), cp)
    _apply(b2, imp, cp)
    return True


class _SinCos(torch.autograd.Function):
    """The build's f32 (sin, cos) (geometry.sincos32); JAX's JVP rules
    d sin = cos, d cos = -sin, on those values."""

    @staticmethod
    def forward(ctx, x):
        s, c = G.sincos32(np.float32(x.item()))
        st, ct = torch.tensor(float(s), dtype=F32), torch.tensor(float(c), dtype=F32)
        ctx.save_for_backward(st, ct)
        return st, ct

    @staticmethod
    def backward(ctx, gs, gc):
        s, c = ctx.saved_tensors
        return gs * c - gc * s


def _rot(v, s, c):  # rotate (cotix/_geometry_utils.py:81-88): [[c,-s],[s,c]] @ v
    return (c * v[0] + (-s) * v[1], s * v[0] + c * v[1])


class _Poly:
    """A world polygon: torch vertices in Polygon.__init__'s clockwise order
    (the permutation is a constant), plus the oracle shape of their values."""

    def __init__(self, verts):
        self.v = verts
        self.np = G.Polygon([(np.float32(x.item()), np.float32(y.item())) for x, y in verts], sort=False)

    def verts(self):
        return self.v

    def edges(self):  # Polygon.edges: (v_k, v_{k-1})
        return [(self.v[k], self.v[k - 1]) for k in range(len(self.v))]


class _Box:
    """A world AABB (lower, upper) with AABB.vertices / edges' corner order."""

    def __init__(self, lo, up):
        self.lo, self.up = lo, up
        self.np = G.AABB((np.float32(lo[0].item()), np.float32(lo[1].item())),
                         (np.float32(up[0].item()), np.float32(up[1].item())))

    def verts(self):
        u, lo = self.up, self.lo
        return [u, (u[0], lo[1]), lo, (lo[0], u[1])]

    def edges(self):
        vs = self.verts()
        return [(vs[k], vs[(k + 1) % 4]) for k in range(4)]


def _world_part(part, p, ang):
    if part.kind == "Circle":
        return (_t(part.radius), (_t(part.position[0]) + p[0], _t(part.position[1]) + p[1]))
    if part.kind == "AABB":
        return _Box((_t(part.lower[0]) + p[0], _t(part.lower[1]) + p[1]),
                    (_t(part.upper[0]) + p[0], _t(part.upper[1]) + p[1]))
    # Polygon.transform: HomogenuousTransformer.forward_vector (t2 == 1), then re-sorted
    s, c = _SinCos.apply(ang)
    ws = [((c * _t(x0) + (-s) * _t(x1)) + p[0] * 1.0, (s * _t(x0) + c * _t(x1)) + p[1] * 1.0)
          for x0, x1 in part.vertices_]
    idx = G.order_clockwise_idx([(np.float32(x.item()), np.float32(y.item())) for x, y in ws])
    return _Poly([ws[k] for k in idx])


# ---- GJK / EPA contacts (cotix/_collisions.py:115-273, cotix/_contacts.py:205-315) ----
def _closest_to_origin(a, b):  # _closest_point_on_edge_to_point(a, b, 0) :156-166
    z = _t(0.0)
    d = _sub(a, b)
    length = d[0] * d[0] + d[1] * d[1]
    if float(length) == 0.0:
        return (z - a[0], z - a[1])
    pb = (z - b[0], z - b[1])
    t = _clip(_dot(pb, d) / length, _t(0.0), _t(1.0))
    proj = (b[0] + d[0] * t, b[1] + d[1] * t)
    return (z - proj[0], z - proj[1])


def _minkowski_point(A, B, pt):
    """The Minkowski point a_i - b_j equal to `pt` (EPA's supports are vertices
    of a polygon or corners of an AABB, chosen by argmax: constants).  Rule,
    shared with the kernel's VJP (cotix_grad.h): the first (i, j), A-major,
    whose difference equals pt."""
    va, vb = A.np.vertices(), B.np.vertices()
    for i, a in enumerate(va):
        for j, b in enumerate(vb):
            if a[0] - b[0] == pt[0] and a[1] - b[1] == pt[1]:
                ta, tb = A.verts()[i], B.verts()[j]
                return (ta[0] - tb[0], ta[1] - tb[1])
    raise AssertionError("EPA edge point is not a Minkowski vertex pair")


def _edge_vs_edge(ea, eb):  # :206-225, the intersecting branch
    p, r = ea[0], _sub(ea[1], ea[0])
    q, s = eb[0], _sub(eb[1], eb[0])
    c = r[0] * s[1] - s[0] * r[1]
    qp = _sub(q, p)
    t = (qp[0] * s[1] - s[0] * qp[1]) / c
    return (p[0] + r[0] * t, p[1] + r[1] * t)


def _contact_from_edges(A, B):
    """:205-267 with the inclusion of each term (vertex containment, edge
    intersection) decided by the oracle on the forward values: constants."""
    acc = (_t(0.0), _t(0.0))
    n = np.float32(0.0)
    for v, vn in zip(A.verts(), A.np.vertices()):
        if B.np.contains(vn):
            acc, n = _add(acc, v), n + np.float32(1.0)
    for v, vn in zip(B.verts(), B.np.vertices()):
        if A.np.contains(vn):
            acc, n = _add(acc, v), n + np.float32(1.0)
    ea_np, eb_np = A.np.edges(), B.np.edges()
    ea_t, eb_t = A.edges(), B.edges()
    for jb in range(len(eb_np)):
        for ia in range(len(ea_np)):
            if not G.vnan(G._edge_vs_edge(ea_np[ia], eb_np[jb])):
                acc, n = _add(acc, _edge_vs_edge(ea_t[ia], eb_t[jb])), n + np.float32(1.0)
    assert n > 0, "contact without a contact point"
    return (acc[0] / float(n), acc[1] / float(n))


def _convex_contact(fname, A, B, d0):
    """polygon_vs_polygon :294-315 / aabb_vs_polygon :270-291, contact branch."""
    nb_ = len(B.np.vertices())
    na_ = 4 if isinstance(A, _Box) else len(A.np.vertices())
    cap = _params.current().epa_max_iters
    iters = min(cap, (4 if isinstance(A, _Box) else na_) + nb_ + 1)
    hit, simplex = G.check_for_collision_convex(A.np, B.np, d0)
    assert hit, "not a contact"
    best = G.epa_best_edge(A.np, B.np, simplex, iters)
    pen = _closest_to_origin(_minkowski_point(A, B, best[0]), _minkowski_point(A, B, best[1]))
    return pen, _contact_from_edges(A, B)


# ---- circle x polygon (cotix/_contacts.py:157-202) ----
# A circle's support is a function of the search direction (Circle.get_support,
# cotix/_convex_shapes.py:22-26: d / |d| * r + c), so jax.grad goes through
# every GJK and EPA step that built the final edge.  Restated in torch with the
# reference's control flow: every decision (GJK's branches, the polygon
# support's argmax, EPA's closest edge and stop test, the contact point's edge)
# is taken by the faithful oracle (geometry.py) on the f32 values of the
# torch tensors -- the same expressions in the same order, so the values are
# bit-identical (asserted) -- and the values are torch ops: the derivative is
# jax.grad's through the executed branches.
def _f(x):
    return np.float32(x.item())


def _fp(p):
    return (_f(p[0]), _f(p[1]))


def _fnormal(a):  # fast_normal (cotix/_geometry_utils.py:30-34)
    return (-a[1], a[0])


def _circle_polygon_contact(circ, P, d0):
    r, c = circ
    poly = P.np

    def mink(d):  # minkowski_diff(circle.get_support, polygon.get_support, d)
        n = _norm(d)
        sa = ((d[0] / n) * r + c[0], (d[1] / n) * r + c[1])
        dn = (-d[0], -d[1])
        dots = [G.dot(v, _fp(dn)) for v in poly.vertices()]
        k = G.argmax(dots)
        sb = P.verts()[k]
        return (sa[0] - sb[0], sa[1] - sb[1])

    def dotf(a, b):
        return G.dot(_fp(a), _fp(b))

    # GJK, _get_collision_simplex (cotix/_collisions.py:20-112)
    s0 = mink((_t(d0[0]), _t(d0[1])))
    s1 = mink((-s0[0], -s0[1]))
    direction = _fnormal(_sub(s1, s0))
    if dotf(direction, (-s1[0], -s1[1])) > 0:
        s0, s1 = s1, s0
    else:
        direction = (-direction[0], -direction[1])
    s2 = mink(direction)
    for _ in range(_params.current().gjk_max_steps):
        c1 = dotf(s2, direction) <= 0
        c2 = dotf(_fnormal(_sub(s2, s0)), (-s2[0], -s2[1])) < 0
        c3 = dotf(_fnormal(_sub(s1, s2)), (-s2[0], -s2[1])) < 0
        if c1 or (c2 and c3):
            break
        cc = s2
        acn, cbn = _fnormal(_sub(cc, s0)), _fnormal(_sub(s1, cc))
        if dotf(acn, (-cc[0], -cc[1])) >= 0:
            s1, direction = cc, acn
        else:
            s0, direction = cc, cbn
        s2 = mink(direction)
    simplex = [s0, s1, s2]
    sn = [_fp(p) for p in simplex]
    assert G.is_point_in_triangle((G.ZERO, G.ZERO), *sn), "circle x polygon: not a contact"
    # EPA, _get_closest_minkowski_diff (cotix/_collisions.py:115-273), 128 iterations (cotix/_contacts.py:162-163)
    iters = _params.current().epa_circle_iters
    z = (_t(0.0), _t(0.0))
    edges = [(z, z)] * (iters + 3)
    edges[0], edges[1], edges[2] = (s0, s1), (s1, s2), (s2, s0)

    def closest(es):
        _, k = G._closest_edge([(_fp(a), _fp(b)) for a, b in es])
        return es[k], k

    best, bei = closest(edges)
    new_point, prev = s2, edges[0]
    i = 0
    for _ in range(iters):
        bf = (_fp(best[0]), _fp(best[1]))
        pf = (_fp(prev[0]), _fp(prev[1]))
        c1 = G.sumsq(G.vsub(bf[0], bf[1])) > np.float32(1e-9)
        c2 = G.cross(bf[0], bf[1]) >= 0
        nrm = G.fast_normal(G.vsub(pf[0], pf[1]))
        nrm = G.vdivs(nrm, G.norm(nrm))
        dd = G.dot(_fp(new_point), nrm)
        edist = G.norm(G._closest_point_on_edge_to_point(pf[0], pf[1], (G.ZERO, G.ZERO)))
        c4 = (dd - edist > np.float32(1e-6)) or (dd <= 0)
        if not (c4 and not G.vnan(bf[0]) and not G.vnan(bf[1]) and c1 and c2):
            break
        n = _fnormal(_sub(best[0], best[1]))
        nn = _norm(n)
        n = (n[0] / nn, n[1] / nn)
        new_point = mink(n)
        edges[bei] = (best[0], new_point)
        edges[i + 3] = (new_point, best[1])
        prev = best
        best, bei = closest(edges)
        i += 1
    best, _ = closest(edges)
    pen = _closest_to_origin(best[0], best[1])
    # the contact point (cotix/_contacts.py:168-197): the polygon edge nearest
    # to the circle's centre, or the centre when it is farther than r
    disps = []
    for a, b in P.edges():
        d = _sub(a, b)
        length = d[0] * d[0] + d[1] * d[1]
        pb = _sub(c, b)
        tt = _clip(_dot(pb, d) / length, _t(0.0), _t(1.0))
        disps.append(_sub(c, (b[0] + d[0] * tt, b[1] + d[1] * tt)))
    dists = [G.sumsq(_fp(dv)) for dv in disps]
    k = G.argmin(dists)
    rf = _f(r)
    cp = c if dists[k] > rf * rf else (c[0] + disps[k][0], c[1] + disps[k][1])
    want = G.circle_vs_polygon(G.Circle(rf, _fp(c)), poly, d0)
    got = (_fp(pen), _fp(cp))
    assert all(np.float32(x).view(np.uint32) == np.float32(y).view(np.uint32)
               for gv, wv in zip(got, want) for x, y in zip(gv, wv)), (got, want)
    return pen, cp


# ---- LunarLander joints (cotix/_lunar_lander.py:145-218) ----
def _lunar_joints(st):
    f05 = np.float32(0.05)
    lander, rleg, lleg = st[0], st[1], st[2]
    sl, cl = _SinCos.apply(lander.ang)
    sr, cr = _SinCos.apply(rleg.ang)
    sll, cll = _SinCos.apply(lleg.ang)

    def k(x, y):
        return (_t(np.float32(x) * f05), _t(np.float32(y) * f05))

    llj1 = _add(_rot(k(P.LEG_AWAY, -P.LEG_DOWN), sl, cl), lander.p)
    llj2 = _add(_rot(k(P.LEG_AWAY, -P.LEG_DOWN + 8), sl, cl), lander.p)
    lj1 = lleg.p
    lj2 = _add(lleg.p, _rot((_t(0.0), _t(0.4)), sll, cll))
    lrj1 = _add(_rot(k(-P.LEG_AWAY, -P.LEG_DOWN), sl, cl), lander.p)
    lrj2 = _add(_rot(k(-P.LEG_AWAY, -P.LEG_DOWN + 8), sl, cl), lander.p)
    rj1 = rleg.p
    rj2 = _add(rleg.p, _rot((_t(0.0), _t(0.4)), sr, cr))

    def fixed(b1, c1, b2, c2):
        dp = _sub(c1, c2)
        dv = _sub(b1.vel_at(c1), b2.vel_at(c2))
        kk = _norm(dv) + float(np.float32(0.1))
        imp = (dp[0] * 1.0 + (dv[0] * kk) * float(f05), dp[1] * 1.0 + (dv[1] * kk) * float(f05))
        _apply(b1, (-imp[0], -imp[1]), c1)
        _apply(b2, imp, c2)

    fixed(lander, llj1, lleg, lj1)
    fixed(lander, llj2, lleg, lj2)
    fixed(lander, lrj1, rleg, rj1)
    fixed(lander, lrj2, rleg, rj2)
    rleg.w = rleg.w * float(np.float32(0.95))
    lleg.w = lleg.w * float(np.float32(0.95))


CONVEX = ("polygon_vs_polygon", "aabb_vs_polygon")


def step_torch(S, a, bodies, trace, dt, action_body, gravity=False, d0=None, joints=False):
    """One step's continuous map S_t [nb,6] -> S_{t+1} given the oracle's
    discrete choices (trace of the same step).  gravity / joints: the
    LunarLander step (examples/test_viz.py:24-44)."""
    nb = S.shape[0]
    dt = float(np.float32(dt))
    st = []
    for b in range(nb):
        p = (S[b, 0] + S[b, 2] * dt, S[b, 1] + S[b, 3] * dt)
        st.append(_B(p, (S[b, 2], S[b, 3]), S[b, 4] + S[b, 5] * dt, S[b, 5], bodies[b]))
    if gravity:
        st[0].v = (st[0].v[0] + 0.0, st[0].v[1] + float(np.float32(P.LL_GRAVITY)))
    if a is not None:
        st[action_body].v = (st[action_body].v[0] + a[0], st[action_body].v[1] + a[1])
    chosen, src = trace["chosen"], trace["src"]
    for i in range(nb):
        j = chosen[i]
        if j == i:
            continue
        fname, (o1b, o1p), (o2b, o2p) = src[i][j]
        s1 = _world_part(bodies[o1b].parts[o1p], st[o1b].p, st[o1b].ang)
        s2 = _world_part(bodies[o2b].parts[o2p], st[o2b].p, st[o2b].ang)
        if fname in CONTACTS:
            s1 = (s1.lo, s1.up) if isinstance(s1, _Box) else s1
            s2 = (s2.lo, s2.up) if isinstance(s2, _Box) else s2
            pen, cp = CONTACTS[fname](s1, s2)
        elif fname in CONVEX:
            pen, cp = _convex_contact(fname, s1, s2, d0)
        elif fname == "circle_vs_polygon":
            pen, cp = _circle_polygon_contact(s1, s2, d0)
        else:
            raise NotImplementedError("%s is not differentiated" % fname)
        resolve(st[i], st[j], pen, cp)
    if joints:
        _lunar_joints(st)
    rows = [torch.stack([b.p[0], b.p[1], b.v[0], b.v[1], b.ang, b.w]) for b in st]
    return torch.stack(rows)


def rollout_grad(make_bodies, S0, key0, actions, w, action_body, d0, dt=P.DT, step=P.robocup_step):
    """Oracle forward (faithful, f32) + torch VJP chain.
    S0 [nb,6] f32, key0 u32[2], actions [T,2] f32, w [nb*6] f32.
    Returns (ret, grad_actions [T,2], grad_S0 [nb,6], states [T+1,nb,6])."""
    T = actions.shape[0]
    bodies = make_bodies()
    for b, row in zip(bodies, S0):
        b.set_dyn(row)
    key = np.asarray(key0, np.uint32)
    states, traces = [np.array([b.dyn() for b in bodies], np.float32)], []
    for t in range(T):
        tr = {}
        bodies, key = step(bodies, key, d0, None, tr, dt, action=actions[t], action_body=action_body)
        states.append(np.array([b.dyn() for b in bodies], np.float32))
        traces.append(tr)
    wm = np.asarray(w, np.float32).reshape(-1, 6)
    ret = np.float32(0.0)
    for t in range(1, T + 1):
        for k in np.flatnonzero(wm.reshape(-1)):
            ret = np.float32(ret + np.float32(wm.reshape(-1)[k]) * states[t].reshape(-1)[k])
    lam = torch.tensor(wm, dtype=F32)
    ga = np.zeros((T, 2), np.float32)
    meta = make_bodies()
    for t in range(T - 1, -1, -1):
        S = torch.tensor(states[t], dtype=F32, requires_grad=True)
        a = torch.tensor(actions[t], dtype=F32, requires_grad=True)
        ll = step is P.lunar_lander_step
        out = step_torch(S, a, meta, traces[t], dt, action_body, gravity=ll, d0=d0, joints=ll)
        o = out.detach().numpy()
        same = (o.view(np.uint32) == states[t + 1].view(np.uint32)) | (np.isnan(o) & np.isnan(states[t + 1]))
        assert same.all(), "torch restatement diverged from the oracle at step %d: %s vs %s" % (
            t, o[~same], states[t + 1][~same])
        gS, gA = torch.autograd.grad(out, (S, a), lam, allow_unused=True)
        ga[t] = gA.numpy() if gA is not None else 0.0
        lam = gS.detach().clone()
        if t >= 1:
            lam = lam + torch.tensor(wm, dtype=F32)
    return ret, ga, lam.numpy(), np.stack(states)
