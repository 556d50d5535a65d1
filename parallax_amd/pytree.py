"""The reference's own body pytrees into a batched World.

cotix builds its scenes as lists of ``AnyBody`` pytrees (cotix/_bodies.py:
135-186) whose ``shape`` is a ``UniversalShape`` (cotix/_universal_shape.py:
16-30) of convex parts -- ``Circle(radius, position)``, ``AABB(lower,
upper)``, ``Polygon``/``Polygon3``..``Polygon6(vertices)`` (cotix/
_convex_shapes.py:10-229) -- e.g. ``RoboCupEnv().bodies`` (cotix/_robocup.py:
124-130) and ``LunarLander(key).bodies`` (cotix/_lunar_lander.py:143).  This
module reads such objects by the reference's class names and field names
only (no import of cotix, equinox or jax), so the reference's constructors
drop in unchanged:

  world = pa.World.from_bodies(RoboCupEnv().bodies, batch=4096)
  world = pa.World.from_bodies(jax.vmap(lambda k: LunarLander(k).bodies)(keys))

Leaves may be Python / NumPy / JAX / torch values; each may carry a leading
batch dimension (a vmapped pytree: stacked leaves), which becomes the
world's env axis.  The part's class name selects the contact-function
registry entry, as the reference's ``_contact_funcs`` is keyed by exact type
(cotix/_colliders.py:21-35).  A polygon's ``vertices`` are taken as stored:
the reference sorts them in ``AbstractPolygon.__init__`` and edits made with
``eqx.tree_at`` keep their order (cotix/_lunar_lander.py:55-72), so the
field already holds the geometry the reference's collider works on.
"""
import numpy as np
import torch

from . import shapes as S
from .bodies import AnyBody
from .shapes import UniversalShape

# the shape registry of the reference, by exact class name
SHAPE_CLASSES = {"Circle": S.Circle, "AABB": S.AABB, "Polygon": S.Polygon, "Polygon3": S.Polygon3,
                 "Polygon4": S.Polygon4, "Polygon5": S.Polygon5, "Polygon6": S.Polygon6}
BODY_FIELDS = ("mass", "inertia", "position", "velocity", "angle", "angular_velocity", "elasticity",
               "friction_coefficient")


def _leaf(x, name):
    """A leaf as a CPU float32 tensor (torch, NumPy, JAX via __array__, numbers)."""
    if isinstance(x, torch.Tensor):
        return x.detach().to("cpu", torch.float32)
    try:
        return torch.from_numpy(np.array(x, dtype=np.float32, copy=True))
    except (TypeError, ValueError) as e:
        raise TypeError("leaf %s is not a float array (%s)" % (name, type(x).__name__)) from e


class _Batch:
    """The leading batch dimension shared by every batched leaf (None: no
    leaf is batched)."""

    def __init__(self, batch):
        self.B = None if batch is None else int(batch)

    def see(self, t, rank, name):
        """t is a leaf whose unbatched rank is `rank`; returns whether it is batched."""
        if t.dim() == rank:
            return False
        if t.dim() != rank + 1:
            raise ValueError("leaf %s has shape %s (expected rank %d or a leading batch dim)"
                             % (name, tuple(t.shape), rank))
        if self.B is None:
            self.B = int(t.shape[0])
        elif t.shape[0] != self.B:
            raise ValueError("leaf %s has batch %d, the others %d" % (name, t.shape[0], self.B))
        return True


def _per_body(t, batched, name):
    """A static parameter (mass, inertia, elasticity, friction): one value per
    body when it is the same in every env (the scene table), else the [B]
    per-env values (a vmapped constructor that varies it, e.g. domain
    randomization: the scene then carries every env's own parameters,
    COTIX_SCENE_PER_ENV_BODY_PARAMS)."""
    if batched:
        v = t.reshape(t.shape[0], -1)
        if v.shape[1] != 1:
            raise ValueError("%s must be one value per body (per env)" % name)
        b = v.view(torch.int32)
        if not bool((b == b[:1]).all()):  # bit-identical in every env: shared
            return v[:, 0].contiguous()
        t = t[0]
    return float(t.reshape(()))


def _geom(p, field, rank, where, batch):
    """A geometry leaf; batched but bit-identical in every env (a vmapped
    constant, e.g. RoboCup's walls): one shared copy, as the kernels read
    shared geometry once for all envs."""
    t = _leaf(getattr(p, field), where + "." + field)
    if batch.see(t, rank, where + "." + field):
        b = t.reshape(t.shape[0], -1).view(torch.int32)
        if bool((b == b[:1]).all()):
            return t[0]
    return t


def _part(p, where, batch):
    cls = type(p).__name__
    if cls not in SHAPE_CLASSES:
        raise TypeError("%s: shape type %s is not in the contact-function registry (%s)"
                        % (where, cls, ", ".join(SHAPE_CLASSES)))
    if cls == "Circle":
        return S.Circle(_geom(p, "radius", 0, where, batch), _geom(p, "position", 1, where, batch))
    if cls == "AABB":
        return S.AABB(_geom(p, "lower", 1, where, batch), _geom(p, "upper", 1, where, batch))
    # the vertices as stored (module docstring)
    return SHAPE_CLASSES[cls](_geom(p, "vertices", 2, where, batch), presorted=True)


def bodies_from_reference(bodies, batch=None):
    """Reference-style body objects -> (parallax_amd AnyBody list, B).

    ``bodies``: a sequence of objects with the AnyBody fields (BODY_FIELDS,
    ``shape.parts``; ``is_area`` optional).  ``batch``: the env count when no
    leaf is batched (default 1); with batched leaves it must match them."""
    if hasattr(bodies, "bodies") and not isinstance(bodies, (list, tuple)):
        bodies = bodies.bodies  # an env object (RoboCupEnv, LunarLander)
    bt = _Batch(batch)
    out = []
    for i, b in enumerate(bodies):
        where = "bodies[%d]" % i
        missing = [f for f in BODY_FIELDS if not hasattr(b, f)]
        if missing or not hasattr(b, "shape") or not hasattr(b.shape, "parts"):
            raise TypeError("%s (%s) lacks the AnyBody fields %s" % (where, type(b).__name__,
                                                                    missing or ["shape.parts"]))
        lv = {f: _leaf(getattr(b, f), where + "." + f) for f in BODY_FIELDS}
        bat = {f: bt.see(lv[f], 1 if f in ("position", "velocity") else 0, where + "." + f) for f in BODY_FIELDS}
        parts = [_part(p, "%s.shape.parts[%d]" % (where, k), bt) for k, p in enumerate(b.shape.parts)]
        if not parts:
            raise ValueError("%s has no shape parts" % where)
        out.append(AnyBody(shape=UniversalShape(*parts),
                           mass=_per_body(lv["mass"], bat["mass"], where + ".mass"),
                           inertia=_per_body(lv["inertia"], bat["inertia"], where + ".inertia"),
                           elasticity=_per_body(lv["elasticity"], bat["elasticity"], where + ".elasticity"),
                           friction_coefficient=_per_body(lv["friction_coefficient"], bat["friction_coefficient"],
                                                          where + ".friction_coefficient"),
                           position=lv["position"], velocity=lv["velocity"], angle=lv["angle"],
                           angular_velocity=lv["angular_velocity"], is_area=bool(getattr(b, "is_area", False))))
    B = 1 if bt.B is None else bt.B
    if batch is not None and int(batch) != B:
        raise ValueError("batch=%d but the leaves carry a batch of %d" % (batch, B))
    return out, B
