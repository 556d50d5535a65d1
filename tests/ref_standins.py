"""TEST INFRASTRUCTURE: stand-ins for the reference's body pytrees.

Minimal classes written for the tests (not the reference's code) that carry
the reference's class names and field names -- AnyBody (cotix/_bodies.py:
135-186), UniversalShape (cotix/_universal_shape.py:16-30), Circle / AABB /
Polygon / Polygon4 / Polygon6 (cotix/_convex_shapes.py) -- with float32
NumPy leaves, as a jax pytree would hold them.  The scenes are filled from
the oracle's restatement of the reference constructors
(oracle/cotix_oracle/physics.py robocup_bodies / lunar_lander_bodies): a
polygon's vertices as the reference stores them (sorted by Polygon.__init__,
or as edited by eqx.tree_at for the legs).  stack() builds a vmapped pytree:
every leaf with a leading batch dimension."""
import numpy as np

F = np.float32


class UniversalShape:
    def __init__(self, *parts):
        self.parts = list(parts)


class Circle:
    def __init__(self, radius, position):
        self.radius, self.position = np.asarray(radius, F), np.asarray(position, F)


class AABB:
    def __init__(self, lower, upper):
        self.upper, self.lower = np.asarray(upper, F), np.asarray(lower, F)


class Polygon:
    def __init__(self, vertices):
        self.vertices = np.asarray(vertices, F)


class Polygon4(Polygon):
    pass


class Polygon6(Polygon):
    pass


class AnyBody:
    def __init__(self, shape, mass=1.0, inertia=1.0, position=(0.0, 0.0), velocity=(0.0, 0.0), angle=0.0,
                 angular_velocity=0.0, elasticity=1.0, friction_coefficient=1.0, is_area=False):
        self.mass, self.inertia = np.asarray(mass, F), np.asarray(inertia, F)
        self.position, self.velocity = np.asarray(position, F), np.asarray(velocity, F)
        self.angle, self.angular_velocity = np.asarray(angle, F), np.asarray(angular_velocity, F)
        self.elasticity, self.friction_coefficient = np.asarray(elasticity, F), np.asarray(friction_coefficient, F)
        self.is_area = is_area
        self.shape = shape


KINDS = {"Circle": Circle, "AABB": AABB, "Polygon": Polygon, "Polygon4": Polygon4, "Polygon6": Polygon6}


def from_oracle(bodies):
    """Oracle bodies (cotix_oracle.physics.Body) -> stand-in pytrees."""
    out = []
    for b in bodies:
        parts = []
        for p in b.parts:
            if p.kind == "Circle":
                parts.append(Circle(p.radius, p.position))
            elif p.kind == "AABB":
                parts.append(AABB(p.lower, p.upper))
            else:
                parts.append(KINDS[p.kind](p.vertices_))
        out.append(AnyBody(UniversalShape(*parts), b.mass, b.inertia, b.position, b.velocity, b.angle,
                           b.angular_velocity, b.elasticity, b.friction_coefficient, b.is_area))
    return out


def stack(scenes):
    """A list of structurally equal stand-in scenes -> one vmapped scene."""
    def leaves(o, names):
        return {n: np.stack([getattr(x, n) for x in o]) for n in names}
    out = []
    for bs in zip(*scenes):
        parts = []
        for ps in zip(*[b.shape.parts for b in bs]):
            cls = type(ps[0])
            p = cls.__new__(cls)
            names = {"Circle": ("radius", "position"), "AABB": ("lower", "upper")}.get(cls.__name__, ("vertices",))
            p.__dict__.update(leaves(ps, names))
            parts.append(p)
        b = AnyBody.__new__(AnyBody)
        b.__dict__.update(leaves(bs, ("mass", "inertia", "position", "velocity", "angle", "angular_velocity",
                                      "elasticity", "friction_coefficient")))
        b.is_area, b.shape = bs[0].is_area, UniversalShape(*parts)
        out.append(b)
    return out
