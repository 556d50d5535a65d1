"""TEST INFRASTRUCTURE ONLY -- CPU oracle, never imported by the product path.

Scalar float32 restatement of cotix's geometry and narrowphase:
  cotix/_geometry_utils.py   (fast_normal, minkowski_diff, order_clockwise,
                              is_point_in_triangle, rotate, HomogenuousTransformer)
  cotix/_convex_shapes.py    (Circle, AABB, Polygon{,4,6}: supports, contains, edges)
  cotix/_collisions.py       (GJK _get_collision_simplex, EPA _get_closest_minkowski_diff)
  cotix/_contacts.py         (ContactInfo and every *_vs_* contact generator)

Numeric conventions, fixed here and in every other
implementation of this path:
  * all arithmetic is IEEE float32, one rounding per operation, no FMA
    contraction, evaluation order = the reference expression's order;
  * min/max/clip propagate NaN (XLA semantics); argmin/argmax return the first
    NaN if any, else the first extremum;
  * sin/cos/atan2 are the deterministic float32 kernels below (Cody-Waite
    reduction + cephes minimax polynomials).  XLA's own f32 kernels are
    unpinned by the reference; the build fixes these so that the oracle, the
    C port and the HIP kernels agree bit for bit.
"""
import numpy as np

from . import params as _params

np.seterr(all="ignore")
F = np.float32
NAN = F(np.nan)
INF = F(np.inf)
ZERO = F(0.0)
ONE = F(1.0)


# ----------------------------------------------------------------------------
# float32 helpers
# ----------------------------------------------------------------------------
def isnan(x):
    return x != x


def fmax(a, b):
    """lax.max: NaN-propagating; ties return the first operand."""
    if isnan(a):
        return a
    if isnan(b):
        return b
    return a if a >= b else b


def fmin(a, b):
    if isnan(a):
        return a
    if isnan(b):
        return b
    return a if a <= b else b


def clip(x, lo, hi):
    """jnp.clip(x, lo, hi) (jax 0.4.x): minimum(hi, maximum(lo, x))."""
    return fmin(hi, fmax(lo, x))


def argmin(vals):
    for k, v in enumerate(vals):
        if isnan(v):
            return k
    best = 0
    for k in range(1, len(vals)):
        if vals[k] < vals[best]:
            best = k
    return best


def argmax(vals):
    for k, v in enumerate(vals):
        if isnan(v):
            return k
    best = 0
    for k in range(1, len(vals)):
        if vals[k] > vals[best]:
            best = k
    return best


def v2(x, y):
    return (F(x), F(y))


def vadd(a, b):
    return (a[0] + b[0], a[1] + b[1])


def vsub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def vneg(a):
    return (-a[0], -a[1])


def vscale(a, s):
    """vector * scalar (jnp broadcasting: each component times s)."""
    return (a[0] * s, a[1] * s)


def vdivs(a, s):
    return (a[0] / s, a[1] / s)


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1]


def cross(a, b):
    """jnp.cross of 2-vectors: a0*b1 - a1*b0."""
    return a[0] * b[1] - a[1] * b[0]


def sumsq(a):
    """jnp.sum(a ** 2) over 2 components."""
    return a[0] * a[0] + a[1] * a[1]


def norm(a):
    return np.sqrt(sumsq(a))


def vnan(a):
    return isnan(a[0]) or isnan(a[1])


def fast_normal(a):
    """cotix/_geometry_utils.py:30-34 (and perpendicular_vector :70-72)."""
    return (-a[1], a[0])


# ----------------------------------------------------------------------------
# deterministic float32 transcendentals (the build's fixed choice)
# ----------------------------------------------------------------------------
_TWO_OVER_PI = F(0.636619772367581343)
_MAGIC = F(12582912.0)  # 1.5 * 2**23: round-to-nearest-even trick
_PIO2_1 = F(1.5703125)
_PIO2_2 = F(4.837512969970703125e-4)
_PIO2_3 = F(7.54978995489188216e-8)
_S0, _S1, _S2 = F(-1.9515295891e-4), F(8.3321608736e-3), F(-1.6666654611e-1)
_C0, _C1, _C2 = F(2.443315711809948e-5), F(-1.388731625493765e-3), F(4.166664568298827e-2)
PI_F = F(3.14159265358979323846)
PIO2_F = F(1.57079632679489661923)
PIO4_F = F(0.785398163397448309616)
_T3P8 = F(2.414213562373095)
_TP8 = F(0.4142135623730950)
_A0, _A1, _A2, _A3 = F(8.05374449538e-2), F(-1.38776856032e-1), F(1.99777106478e-1), F(-3.33329491539e-1)


def _sin_poly(r):
    z = r * r
    return (((_S0 * z + _S1) * z + _S2) * z) * r + r


def _cos_poly(r):
    z = r * r
    return ((((_C0 * z + _C1) * z + _C2) * z) * z - F(0.5) * z) + ONE


def sincos32(x):
    """Returns (sin x, cos x) in float32.  Quadrant k = rint(x*2/pi) by the
    1.5*2^23 trick, r = ((x - k*P1) - k*P2) - k*P3, cephes polynomials on
    |r| <= pi/4."""
    x = F(x)
    if isnan(x) or np.isinf(x):
        return NAN, NAN
    t = x * _TWO_OVER_PI
    k = (t + _MAGIC) - _MAGIC
    r = ((x - k * _PIO2_1) - k * _PIO2_2) - k * _PIO2_3
    s = _sin_poly(r)
    c = _cos_poly(r)
    q = int(k) & 3
    if q == 0:
        return s, c
    if q == 1:
        return c, -s
    if q == 2:
        return -s, -c
    return -c, s


def _atan01(t):
    """cephes atanf on t in [0, 1]."""
    if t > _TP8:
        y0 = PIO4_F
        t = (t - ONE) / (t + ONE)
    else:
        y0 = ZERO
    z = t * t
    p = ((((_A0 * z + _A1) * z + _A2) * z + _A3) * z) * t + t
    return y0 + p


def atan2_32(y, x):
    y = F(y)
    x = F(x)
    if isnan(x) or isnan(y):
        return NAN
    if y == ZERO:
        if x > ZERO or (x == ZERO and not np.signbit(x)):
            return y
        return -PI_F if np.signbit(y) else PI_F
    if x == ZERO:
        return -PIO2_F if y < ZERO else PIO2_F
    ax = F(abs(x))
    ay = F(abs(y))
    if ay <= ax:
        r = _atan01(ay / ax)
    else:
        r = PIO2_F - _atan01(ax / ay)
    if x < ZERO:
        r = PI_F - r
    return -r if y < ZERO else r


def _sort_key(v):
    """lax.sort float order: -0 == +0, every NaN after +inf (all NaN equal)."""
    if isnan(v):
        return (1, 0.0)
    return (0, float(v) + 0.0)


def order_clockwise_idx(verts):
    """cotix/_geometry_utils.py:60-67: subtract the (sequentially summed) mean,
    atan2, stable argsort."""
    n = len(verts)
    sx = ZERO
    sy = ZERO
    for v in verts:
        sx = sx + v[0]
        sy = sy + v[1]
    mx = sx / F(n)
    my = sy / F(n)
    ang = [atan2_32(v[1] - my, v[0] - mx) for v in verts]
    return sorted(range(n), key=lambda k: _sort_key(ang[k]))  # Python sort is stable


def order_clockwise(verts):
    return [verts[k] for k in order_clockwise_idx(verts)]


def rotate(vec, angle):
    """cotix/_geometry_utils.py:81-88: [[c,-s],[s,c]] @ v."""
    s, c = sincos32(angle)
    return (c * vec[0] + (-s) * vec[1], s * vec[0] + c * vec[1])


class Transformer:
    """HomogenuousTransformer (cotix/_geometry_utils.py:91-142).  Only the
    forward map and shift() are on the hot path (the inverse is never read)."""

    def __init__(self, position, angle):
        self.position = (F(position[0]), F(position[1]))
        self.angle = F(angle)
        self.sin, self.cos = sincos32(self.angle)

    def forward_vector(self, x):
        """M @ [x0, x1, 1] then divide by the homogeneous coordinate
        (cotix/_geometry_utils.py:134-138)."""
        c, s = self.cos, self.sin
        px, py = self.position
        t0 = (c * x[0] + (-s) * x[1]) + px * ONE
        t1 = (s * x[0] + c * x[1]) + py * ONE
        t2 = (ZERO * x[0] + ZERO * x[1]) + ONE * ONE
        return (t0 / t2, t1 / t2)

    def shift(self):
        return self.position


# ----------------------------------------------------------------------------
# shapes (cotix/_convex_shapes.py)
# ----------------------------------------------------------------------------
class Circle:
    kind = "Circle"

    def __init__(self, radius, position):
        self.radius = F(radius)
        self.position = (F(position[0]), F(position[1]))

    def support(self, d):  # :22-26
        n = norm(d)
        nd = (d[0] / n, d[1] / n)
        return (nd[0] * self.radius + self.position[0], nd[1] * self.radius + self.position[1])

    def contains(self, p, eps=1e-6):  # :28-29
        r = self.radius + F(eps)
        return bool(sumsq(vsub(p, self.position)) <= r * r)

    def center(self):
        return self.position

    def transform(self, T):  # :37-41 (translate only)
        return Circle(self.radius, vadd(self.position, T.shift()))

    def move(self, delta):
        return Circle(self.radius, vadd(self.position, delta))


class AABB:
    kind = "AABB"

    def __init__(self, lower, upper):
        self.lower = (F(lower[0]), F(lower[1]))
        self.upper = (F(upper[0]), F(upper[1]))

    def support(self, d):  # :62-66
        return (self.upper[0] if d[0] >= ZERO else self.lower[0],
                self.upper[1] if d[1] >= ZERO else self.lower[1])

    def center(self):  # :79-80
        return ((self.lower[0] + self.upper[0]) / F(2.0), (self.lower[1] + self.upper[1]) / F(2.0))

    def vertices(self):  # :95-103
        u, lo = self.upper, self.lower
        return [u, (u[0], lo[1]), lo, (lo[0], u[1])]

    def edges(self):  # :82-93
        vs = self.vertices()
        return [(vs[0], vs[1]), (vs[1], vs[2]), (vs[2], vs[3]), (vs[3], vs[0])]

    def contains(self, p, eps=1e-6):  # :105-106
        e = F(eps)
        return bool((p[0] >= self.lower[0] - e) and (p[1] >= self.lower[1] - e)
                    and (p[0] <= self.upper[0] + e) and (p[1] <= self.upper[1] + e))

    def transform(self, T):  # :113-117 (translate only)
        s = T.shift()
        return AABB(vadd(self.lower, s), vadd(self.upper, s))

    def move(self, delta):
        return AABB(vadd(self.lower, delta), vadd(self.upper, delta))


class Polygon:
    """AbstractPolygon (cotix/_convex_shapes.py:136-194).  ``kind`` is the
    exact registry type: Polygon, Polygon3..Polygon6 by construction."""

    def __init__(self, vertices, kind=None, sort=True):
        vs = [(F(v[0]), F(v[1])) for v in vertices]
        self.vertices_ = order_clockwise(vs) if sort else vs
        self.kind = kind or "Polygon%d" % len(vs)

    def support(self, d):  # :149-155
        if vnan(d):
            return (NAN, NAN)
        dots = [dot(v, d) for v in self.vertices_]
        return self.vertices_[argmax(dots)]

    def center(self):
        n = len(self.vertices_)
        sx, sy = ZERO, ZERO
        for v in self.vertices_:
            sx, sy = sx + v[0], sy + v[1]
        return (sx / F(n), sy / F(n))

    def vertices(self):
        return list(self.vertices_)

    def edges(self):  # :160-163: edge k = (v_k, v_{k-1})
        vs = self.vertices_
        return [(vs[k], vs[k - 1]) for k in range(len(vs))]

    def contains(self, p):  # :168-175
        dots = []
        for e0, e1 in self.edges():
            d = dot(vsub(p, e0), fast_normal(vsub(e0, e1)))
            dots.append(F(np.sign(d)))
        return all(bool(d == dots[0]) for d in dots)

    def transform(self, T):  # :181-187 (affine, then re-sorted by __init__)
        return Polygon([T.forward_vector(v) for v in self.vertices_], kind=self.kind)

    def move(self, delta):
        return Polygon([vadd(v, delta) for v in self.vertices_], kind=self.kind)


# ----------------------------------------------------------------------------
# GJK / EPA (cotix/_collisions.py)
# ----------------------------------------------------------------------------
def minkowski_diff(a, b, d):
    """cotix/_geometry_utils.py:49-57."""
    return vsub(a.support(d), b.support(vneg(d)))


def is_point_in_triangle(pt, v1, v2, v3):
    """cotix/_geometry_utils.py:12-27."""
    def sign(p1, p2, p3):
        return (p1[0] - p3[0]) * (p2[1] - p3[1]) - (p2[0] - p3[0]) * (p1[1] - p3[1])

    d1, d2, d3 = sign(pt, v1, v2), sign(pt, v2, v3), sign(pt, v3, v1)
    has_neg = (d1 < 0) or (d2 < 0) or (d3 < 0)
    has_pos = (d1 > 0) or (d2 > 0) or (d3 > 0)
    return not (has_neg and has_pos)


GJK_MAX_STEPS = 32


def gjk_simplex(a, b, d0):
    """_get_collision_simplex (cotix/_collisions.py:20-112)."""
    s0 = minkowski_diff(a, b, d0)
    s1 = minkowski_diff(a, b, vneg(s0))
    direction = fast_normal(vsub(s1, s0))
    if dot(direction, vneg(s1)) > 0:  # :47-53
        s0, s1 = s1, s0
    else:
        direction = vneg(direction)
    s2 = minkowski_diff(a, b, direction)
    steps = 0
    while steps < _params.current().gjk_max_steps:  # eqx while_loop(max_steps=32), :100-102
        c1 = dot(s2, direction) <= 0
        c2 = dot(fast_normal(vsub(s2, s0)), vneg(s2)) < 0
        c3 = dot(fast_normal(vsub(s1, s2)), vneg(s2)) < 0
        if c1 or (c2 and c3):
            break
        c = s2
        ac_normal = fast_normal(vsub(c, s0))
        cb_normal = fast_normal(vsub(s1, c))
        if dot(ac_normal, vneg(c)) >= 0:  # :71-75
            s1 = c
            direction = ac_normal
        else:
            s0 = c
            direction = cb_normal
        s2 = minkowski_diff(a, b, direction)
        steps += 1
    z = (ZERO, ZERO)
    if is_point_in_triangle((ZERO, ZERO), s0, s1, s2):  # :105-110
        return [s0, s1, s2]
    return [z, z, z]


def check_for_collision_convex(a, b, d0):
    """cotix/_collisions.py:277-310 (initial_direction NaN -> random_direction
    of PRNGKey(1), a constant)."""
    s = gjk_simplex(a, b, d0)
    area = cross(vsub(s[1], s[0]), vsub(s[2], s[0]))
    allzero = all(v[0] == 0 and v[1] == 0 for v in s)
    anynan = any(vnan(v) for v in s)
    if allzero or anynan or area == 0:
        return False, [(NAN, NAN)] * 3
    return True, s


def _closest_point_on_edge_to_point(a, b, point):  # :156-166
    length = sumsq(vsub(a, b))
    if length == 0:
        return vsub(point, a)
    t = dot(vsub(point, b), vsub(a, b)) / length
    t = clip(t, ZERO, ONE)
    proj = vadd(b, vscale(vsub(a, b), t))
    return vsub(point, proj)


def _displacement_to_origin(a, b):  # :137-154
    if a[0] == 0 and a[1] == 0 and b[0] == 0 and b[1] == 0:
        return (INF, INF)
    point = (ZERO, ZERO)
    length = sumsq(vsub(a, b))
    t = dot(vsub(point, b), vsub(a, b)) / length
    t = clip(t, ZERO, ONE)
    proj = vadd(b, vscale(vsub(a, b), t))
    disp = vsub(point, proj)
    return vneg(a) if length == 0 else disp


def _closest_edge(edges):  # :171-175
    dists = [sumsq(_displacement_to_origin(e[0], e[1])) for e in edges]
    k = argmin(dists)
    return edges[k], k


def epa(a, b, simplex, iters):
    """_get_closest_minkowski_diff (cotix/_collisions.py:115-273)."""
    best = epa_best_edge(a, b, simplex, iters)
    return _closest_point_on_edge_to_point(best[0], best[1], (ZERO, ZERO))


def epa_best_edge(a, b, simplex, iters):
    """EPA's final closest polytope edge (two Minkowski points).  The scan of
    ``iters`` conditional bodies stops at the first false condition: the state
    is a fixed point afterwards (value-identical early exit)."""
    z = (ZERO, ZERO)
    edges = [(z, z)] * (iters + 3)
    edges[0] = (simplex[0], simplex[1])
    edges[1] = (simplex[1], simplex[2])
    edges[2] = (simplex[2], simplex[0])
    best, bei = _closest_edge(edges)
    new_point = simplex[2]
    prev = edges[0]
    i = 0
    for _ in range(iters):
        # cond_fn :178-212
        c1 = sumsq(vsub(best[0], best[1])) > F(1e-9)
        c2 = cross(best[0], best[1]) >= 0
        nrm = fast_normal(vsub(prev[0], prev[1]))
        nrm = vdivs(nrm, norm(nrm))
        d = dot(new_point, nrm)
        edist = norm(_closest_point_on_edge_to_point(prev[0], prev[1], (ZERO, ZERO)))
        c4 = (d - edist > F(1e-6)) or (d <= 0)
        if not (c4 and not vnan(best[0]) and not vnan(best[1]) and c1 and c2):
            break
        # body_fn :214-236
        nrm = fast_normal(vsub(best[0], best[1]))
        nrm = vdivs(nrm, norm(nrm))
        new_point = minkowski_diff(a, b, nrm)
        edges[bei] = (best[0], new_point)
        edges[i + 3] = (new_point, best[1])
        prev = best
        best, bei = _closest_edge(edges)
        i += 1
    best, _ = _closest_edge(edges)
    return best


# ----------------------------------------------------------------------------
# contact generators (cotix/_contacts.py)
# ----------------------------------------------------------------------------
NAN_CONTACT = ((ZERO, ZERO), (NAN, NAN))  # ContactInfo.nan(), :19-21


def contact_isnan(c):
    return vnan(c[1])


class ErrorFlag:
    """Collects ``eqx.error_if`` trips (EQX_ON_ERROR=nan semantics: the
    guarded value becomes NaN and a flag is raised)."""

    CIRCLE_AABB_CCP = 1

    def __init__(self):
        self.bits = 0


def circle_vs_circle(a, b, err=None):  # :30-58
    delta = vsub(a.position, b.position)
    distance = norm(delta)
    direction = (ONE, ZERO) if distance == 0 else vdivs(delta, distance)
    pen = vscale(direction, fmin(distance - (a.radius + b.radius), ZERO))
    cp = vdivs(vadd(vadd(b.position, vscale(direction, b.radius - a.radius)), a.position), F(2.0))
    if not (dot(vsub(a.position, cp), vsub(b.position, cp)) <= 0):
        cp = b.position if a.contains(b.position) else a.position
    if distance <= a.radius + b.radius:
        return (vneg(pen), cp)
    return NAN_CONTACT


def aabb_vs_aabb(a, b, err=None, eps=1e-8):  # :61-96
    below = a.upper[1] <= b.lower[1]
    above = a.lower[1] >= b.upper[1]
    left = a.upper[0] <= b.lower[0]
    right = a.lower[0] >= b.upper[0]
    if below or left or above or right:
        return NAN_CONTACT
    me = -F(eps)
    depths = [fmax(a.upper[1] - b.lower[1], me), fmax(b.upper[1] - a.lower[1], me),
              fmax(a.upper[0] - b.lower[0], me), fmax(b.upper[0] - a.lower[0], me)]
    dirs = [(0, -1), (0, 1), (-1, 0), (1, 0)]
    k = argmin(depths)
    md = fmax(ZERO, depths[k])  # clip(a_min=0)
    pen = (md * F(dirs[k][0]), md * F(dirs[k][1]))
    mu = (fmin(a.upper[0], b.upper[0]), fmin(a.upper[1], b.upper[1]))
    ml = (fmax(a.lower[0], b.lower[0]), fmax(a.lower[1], b.lower[1]))
    return (pen, vdivs(vadd(mu, ml), F(2.0)))


def circle_vs_aabb(a, b, err=None, eps=1e-6):  # :99-154
    bc = b.center()
    disp = vsub(a.center(), bc)
    lo = vsub(b.lower, bc)
    hi = vsub(b.upper, bc)
    cd = (clip(disp[0], lo[0], hi[0]), clip(disp[1], lo[1], hi[1]))
    ccp = vadd(bc, cd)
    if not b.contains(ccp):  # eqx.error_if :105-107
        if err is not None:
            err.bits |= ErrorFlag.CIRCLE_AABB_CCP
        ccp = (NAN, NAN)
    vs = [b.lower, (b.lower[0], b.upper[1]), b.upper, (b.upper[0], b.lower[1])]
    e = F(eps)
    perfect_vertex = any(bool(norm(vsub(v, ccp)) < e) for v in vs)
    if not a.contains(ccp):
        return NAN_CONTACT
    if perfect_vertex:  # circle_dir_move :120-125
        d = vsub(ccp, a.position)
        dn = vdivs(d, norm(d))
        return (vneg(vsub(vadd(a.position, vscale(dn, a.radius)), ccp)), ccp)
    r = a.radius  # aligned_move :127-148
    shifts = [(a.position[1] + r) - b.lower[1], b.upper[1] - (a.position[1] - r),
              (a.position[0] + r) - b.lower[0], b.upper[0] - (a.position[0] - r)]
    dirs = [(0, 1), (0, -1), (1, 0), (-1, 0)]
    k = argmin(shifts)
    ns = -shifts[k]
    return ((ns * F(dirs[k][0]), ns * F(dirs[k][1])), ccp)


def _edge_point_displacement(edge, point):  # :168-184
    a, b = edge
    if a[0] == 0 and a[1] == 0 and b[0] == 0 and b[1] == 0:
        return (INF, INF)
    length = sumsq(vsub(a, b))
    t = dot(vsub(point, b), vsub(a, b)) / length
    t = clip(t, ZERO, ONE)
    proj = vadd(b, vscale(vsub(a, b), t))
    return vsub(point, proj)


def circle_vs_polygon(circle, polygon, d0, err=None):  # :157-202
    exists, simplex = check_for_collision_convex(circle, polygon, d0)
    if not exists:
        return NAN_CONTACT
    pen = epa(circle, polygon, simplex, _params.current().epa_circle_iters)
    disps = [_edge_point_displacement(e, circle.position) for e in polygon.edges()]
    dists = [sumsq(d) for d in disps]
    k = argmin(dists)
    cp = vadd(circle.position, disps[k])
    if dists[k] > circle.radius * circle.radius:
        cp = circle.position
    return (pen, cp)


def _edge_vs_edge(ea, eb):  # :206-225
    p = ea[0]
    r = vsub(ea[1], ea[0])
    q = eb[0]
    s = vsub(eb[1], eb[0])

    def crs(u, v):
        return u[0] * v[1] - v[0] * u[1]

    c = crs(r, s)
    t = crs(vsub(q, p), s) / c
    u = crs(vsub(q, p), r) / c
    if c != 0 and t >= 0 and t <= 1 and u >= 0 and u <= 1:
        return vadd(p, vscale(r, t))
    return (NAN, NAN)


def contact_from_edges(edges_a, verts_a, in_a, edges_b, verts_b, in_b):  # :205-267
    inters = [_edge_vs_edge(ea, eb) for eb in edges_b for ea in edges_a]
    n = ZERO
    acc = (ZERO, ZERO)
    for v in verts_a:
        if in_b(v):
            acc = vadd(acc, v)
            n = n + ONE
    for v in verts_b:
        if in_a(v):
            acc = vadd(acc, v)
            n = n + ONE
    for x in inters:
        if not vnan(x):
            acc = vadd(acc, x)
            n = n + ONE
    if n > 0:
        return vdivs(acc, n)
    return (NAN, NAN)


def aabb_vs_polygon(aabb, polygon, d0, err=None):  # :270-291
    iters = min(_params.current().epa_max_iters, 4 + len(polygon.vertices_) + 1)
    exists, simplex = check_for_collision_convex(aabb, polygon, d0)
    if not exists:
        return NAN_CONTACT
    pen = epa(aabb, polygon, simplex, iters)
    cp = contact_from_edges(aabb.edges(), aabb.vertices(), aabb.contains,
                            polygon.edges(), polygon.vertices(), polygon.contains)
    return (pen, cp)


def polygon_vs_polygon(pa, pb, d0, err=None):  # :294-315
    iters = min(_params.current().epa_max_iters, len(pa.vertices_) + len(pb.vertices_) + 1)
    exists, simplex = check_for_collision_convex(pa, pb, d0)
    if not exists:
        return NAN_CONTACT
    pen = epa(pa, pb, simplex, iters)
    cp = contact_from_edges(pa.edges(), pa.vertices(), pa.contains,
                            pb.edges(), pb.vertices(), pb.contains)
    return (pen, cp)


# _contact_funcs (cotix/_colliders.py:21-35), keyed by exact type names.
CONTACT_FUNCS = {
    ("AABB", "AABB"): "aabb_vs_aabb",
    ("Circle", "Circle"): "circle_vs_circle",
    ("Circle", "AABB"): "circle_vs_aabb",
    ("Polygon", "Polygon"): "polygon_vs_polygon",
    ("AABB", "Polygon"): "aabb_vs_polygon",
    ("Circle", "Polygon"): "circle_vs_polygon",
    ("Circle", "Polygon4"): "circle_vs_polygon",
    ("Circle", "Polygon6"): "circle_vs_polygon",
    ("AABB", "Polygon4"): "aabb_vs_polygon",
    ("AABB", "Polygon6"): "aabb_vs_polygon",
    ("Polygon4", "Polygon4"): "polygon_vs_polygon",
    ("Polygon4", "Polygon6"): "polygon_vs_polygon",
    ("Polygon6", "Polygon6"): "polygon_vs_polygon",
}


def run_contact(fname, a, b, d0, err=None):
    if fname == "aabb_vs_aabb":
        return aabb_vs_aabb(a, b, err)
    if fname == "circle_vs_circle":
        return circle_vs_circle(a, b, err)
    if fname == "circle_vs_aabb":
        return circle_vs_aabb(a, b, err)
    if fname == "circle_vs_polygon":
        return circle_vs_polygon(a, b, d0, err)
    if fname == "aabb_vs_polygon":
        return aabb_vs_polygon(a, b, d0, err)
    if fname == "polygon_vs_polygon":
        return polygon_vs_polygon(a, b, d0, err)
    raise KeyError(fname)
