"""TEST INFRASTRUCTURE ONLY -- body-level operators of UniversalShape
(cotix/_universal_shape.py:32-132) restated over the oracle's geometry.

wrap_local_support (:32-45) computes inverse_direction(direction) and drops
the result (:38): the part's LOCAL support is taken in the global direction and
mapped forward by the body transform.  collides_with keeps the first colliding
part pair's simplex (:87-107); penetration_depth runs EPA for 48 iterations
(:121-132).  possibly_collides_with (:109-110) calls AABB.of_universal and
AABB.collides, which do not exist in the reference; the build defines the
body's AABB as AABB.of (cotix/_convex_shapes.py:68-77) of its global support
(get_global_support, :47-59) and the overlap test as the negation of
aabb_vs_aabb's separation test (cotix/_contacts.py:62-65)."""
from . import geometry as G
from . import params as _params

F = G.F
NAN = G.NAN


class WrappedPart:
    def __init__(self, part, tf):
        self.part, self.tf = part, tf

    def support(self, d):
        return self.tf.forward_vector(self.part.support(d))


def penetrates_with(body_a, body_b, d0):
    """-> (collides, penetration vector)."""
    ta, tb = body_a.transformer(), body_b.transformer()
    hit, first, simplex = False, None, None
    for pa in body_a.parts:
        for pb in body_b.parts:
            wa, wb = WrappedPart(pa, ta), WrappedPart(pb, tb)
            res, s = G.check_for_collision_convex(wa, wb, d0)
            if res and not hit:
                first, simplex = (wa, wb), s
            hit = hit or res
    if not hit:
        return False, (G.ZERO, G.ZERO)
    return True, G.epa(first[0], first[1], simplex, _params.current().epa_body_iters)


def body_aabb(body):
    """-> ((lo.x, lo.y, up.x, up.y), error bits)."""
    tf = body.transformer()
    parts = [WrappedPart(p, tf) for p in body.parts]

    def gsupport(d):
        sups = [w.support(d) for w in parts]
        return sups[G.argmax([G.dot(s, d) for s in sups])]

    one, z = F(1.0), G.ZERO
    xmin = gsupport((-one, z))[0]
    ymin = gsupport((z, -one))[1]
    xmax = gsupport((one, z))[0]
    ymax = gsupport((z, one))[1]
    err = 0
    if xmax <= xmin:
        err, xmax = err | 2, NAN
    if ymax <= ymin:
        err, ymax = err | 2, NAN
    return (xmin, ymin, xmax, ymax), err
