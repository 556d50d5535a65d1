"""Convex shapes and the composite UniversalShape (host-side descriptions).

Mirrors cotix/_convex_shapes.py (Circle :10-47, AABB :50-133, Polygon{,3..6}
:136-229) and cotix/_universal_shape.py:16-69.  A shape holds its LOCAL
geometry; world-frame transforms (translate-only for Circle/AABB, affine +
re-sort for polygons) happen on the device every step.  Geometry leaves may
be Python numbers / sequences (shared by every env) or float32 tensors with
a leading batch dimension (per-env geometry, e.g. LunarLander terrain).
"""
import torch

from . import _ffi


def _f32(x):
    return torch.as_tensor(x, dtype=torch.float32)


class AbstractConvexShape:
    type_id = None

    def geom_floats(self):
        raise NotImplementedError

    def local_geometry(self):
        """float32 tensor [..., geom_floats]: per-env when batched."""
        raise NotImplementedError


class Circle(AbstractConvexShape):
    type_id = _ffi.CIRCLE

    def __init__(self, radius, position):
        self.radius = _f32(radius)
        self.position = _f32(position)

    def geom_floats(self):
        return 4

    def local_geometry(self):
        """(radius, cx, cy, 0): circles are padded to the AABB's 4 floats."""
        lead = torch.broadcast_shapes(self.radius.shape, self.position.shape[:-1])
        r = self.radius.expand(lead).unsqueeze(-1)
        return torch.cat([r, self.position.expand(*lead, 2), torch.zeros_like(r)], dim=-1)


class AABB(AbstractConvexShape):
    type_id = _ffi.AABB

    def __init__(self, lower, upper):
        self.lower = _f32(lower)
        self.upper = _f32(upper)

    def geom_floats(self):
        return 4

    def local_geometry(self):
        lo, up = torch.broadcast_tensors(self.lower, self.upper)
        return torch.cat([lo, up], dim=-1)


class AbstractPolygon(AbstractConvexShape):
    """Convex polygon; ``vertices`` [..., n, 2].  Like the reference's
    __init__ (order_clockwise, cotix/_convex_shapes.py:143-144) the vertices
    are sorted -- on the device, when the world uploads its geometry --
    unless ``presorted`` (the reference's eqx.tree_at edits bypass __init__,
    e.g. cotix/_lunar_lander.py:55-72)."""

    type_id = _ffi.POLYGON
    nverts = None

    def __init__(self, vertices, presorted=False):
        self.vertices = _f32(vertices)
        if self.nverts is not None and self.vertices.shape[-2] != self.nverts:
            raise ValueError("%s needs %d vertices" % (type(self).__name__, self.nverts))
        if not 3 <= self.vertices.shape[-2] <= 8:
            raise ValueError("polygons have 3..8 vertices on this path")
        self.presorted = presorted

    def geom_floats(self):
        return 2 * self.vertices.shape[-2]

    def local_geometry(self):
        return self.vertices.reshape(*self.vertices.shape[:-2], -1)


class Polygon(AbstractPolygon):
    type_id = _ffi.POLYGON


class Polygon3(AbstractPolygon):
    type_id, nverts = _ffi.POLYGON3, 3


class Polygon4(AbstractPolygon):
    type_id, nverts = _ffi.POLYGON4, 4


class Polygon5(AbstractPolygon):
    type_id, nverts = _ffi.POLYGON5, 5


class Polygon6(AbstractPolygon):
    type_id, nverts = _ffi.POLYGON6, 6


class UniversalShape:
    """Composite shape: a list of convex parts (cotix/_universal_shape.py:16-30)."""

    def __init__(self, *shapes):
        self.parts = list(shapes)
