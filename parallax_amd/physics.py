"""The reference's operator/plugin surface for the hot path, over Worlds.

  ExplicitEulerPhysics.step(bodies, dt) -> (bodies, self)     cotix/_physics_solvers.py:16-33
  RandomizedCollider.resolve(bodies, rkey) -> bodies          cotix/_colliders.py:74-351
  SimpleConstraintSolver(loops).solve(bodies, constraints)    cotix/_constraint_solvers.py:4-17
  contact_funcs[(Ta, Tb)](a, b) -> ContactInfo (batched)      cotix/_colliders.py:21-35
  resolve_collision(b1, b2, contact) (batched)                cotix/_collision_resolution.py:52-151

``bodies`` is a World (the batched body list); operators update it in place
on the device and return it, so the reference's functional call sites
(``new_bodies, _ = physics.step(bodies, dt)``) read the same.
"""
import numpy as np
import torch

from . import _ffi
from .shapes import AABB, Circle, Polygon, Polygon4, Polygon6


class AbstractPhysicsSolver:
    def step(self, bodies, dt):
        raise NotImplementedError


class ExplicitEulerPhysics(AbstractPhysicsSolver):
    def step(self, bodies, dt=1e-2):
        bodies.euler(dt)
        return bodies, self


class AbstractCollider:
    def resolve(self, bodies, *args, **kwargs):
        raise NotImplementedError


class RandomizedCollider(AbstractCollider):
    def resolve(self, bodies, rkey=None, collision_callback=None):
        """rkey: [B, 2] int32 keys (default: the world's own keys)."""
        bodies.collide(rkey)
        return bodies


class SimpleConstraintSolver:
    """No constraint class exists in the reference (grep: only
    cotix/_constraint_solvers.py:8-16): with an empty list the solve is the
    identity SoA round trip."""

    def __init__(self, loops=1):
        self.loops = loops

    def solve(self, bodies, constraints):
        for _ in range(self.loops):
            for c in constraints:
                bodies = c.apply(bodies)
        return bodies


class ContactInfo:
    """Batched ContactInfo (cotix/_contacts.py:11-27): NaN contact_point = none."""

    def __init__(self, penetration_vector, contact_point):
        self.penetration_vector = penetration_vector
        self.contact_point = contact_point

    def isnan(self):
        return torch.isnan(self.contact_point).any(-1)


def shape_rows(shapes_geometry, kind, nverts=0):
    """Pack world-frame geometry [n, k] into the [n, 18] operator layout."""
    n = shapes_geometry.shape[0]
    out = torch.zeros(n, 18, dtype=torch.float32, device=shapes_geometry.device)
    out[:, 0] = kind
    out[:, 1] = nverts
    out[:, 2:2 + shapes_geometry.shape[1]] = shapes_geometry
    return out


KIND = {Circle: 0, AABB: 1}


def _params_ref(params):
    import ctypes
    return None if params is None else ctypes.byref(params.c_struct())


def run_contacts(fn, a_rows, b_rows, params=None):
    """cotix_contacts_ex over [n, 18] shape rows -> (ContactInfo, err[n]);
    params: parallax_amd.Params (GJK steps, EPA iterations, the GJK start
    direction's PRNG layout), None: the reference's literals."""
    n = a_rows.shape[0]
    out = torch.empty(n, 4, dtype=torch.float32, device=a_rows.device)
    err = torch.zeros(n, dtype=torch.int32, device=a_rows.device)
    _ffi.check(_ffi.lib.cotix_contacts_ex(fn, n, _ffi.ptr(a_rows.contiguous()), _ffi.ptr(b_rows.contiguous()),
                                          _ffi.ptr(out), _ffi.ptr(err), _params_ref(params),
                                          _ffi.stream_ptr(a_rows.device)), "cotix_contacts_ex")
    return ContactInfo(out[:, 0:2], out[:, 2:4]), err


def check_for_collision_convex(a_rows, b_rows, params=None, initial_direction=None, key=None):
    """check_for_collision_convex(a.get_support, b.get_support,
    initial_direction, key) (cotix/_collisions.py:277-310) over [n, 18] shape
    rows: (hit bool [n], simplex f32 [n, 3, 2]) -- NaN * simplex where there
    is no collision.  initial_direction: None (the default [nan, nan]) or f32
    [n, 2] / [2]; key: None (PRNGKey(1)) or u32 / i32 [n, 2] / [2] keys; the
    start direction is random_direction(key) blended 0.1 / 0.9 with a non-NaN
    initial_direction, as the reference."""
    n = a_rows.shape[0]
    dev = a_rows.device
    hit = torch.empty(n, dtype=torch.int32, device=dev)
    simplex = torch.empty(n, 3, 2, dtype=torch.float32, device=dev)
    init = None if initial_direction is None else \
        torch.as_tensor(initial_direction, dtype=torch.float32, device=dev).expand(n, 2).contiguous()
    if key is None:
        keys = None
    else:
        kt = key if isinstance(key, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(np.asarray(key, dtype=np.uint32)).view(np.int32))
        keys = kt.to(dev, torch.int32).expand(n, 2).contiguous()
    _ffi.check(_ffi.lib.cotix_gjk_ex(n, _ffi.ptr(a_rows.contiguous()), _ffi.ptr(b_rows.contiguous()), _ffi.ptr(init),
                                     _ffi.ptr(keys), _ffi.ptr(hit), _ffi.ptr(simplex), _params_ref(params),
                                     _ffi.stream_ptr(dev)), "cotix_gjk_ex")
    return hit.bool(), simplex


def compute_penetration_vector_convex(a_rows, b_rows, simplex, solver_iterations=48):
    """compute_penetration_vector_convex (cotix/_collisions.py:313-329): EPA
    from the given simplices [n, 3, 2] -> penetration f32 [n, 2]."""
    n = a_rows.shape[0]
    pen = torch.empty(n, 2, dtype=torch.float32, device=a_rows.device)
    _ffi.check(_ffi.lib.cotix_epa(n, _ffi.ptr(a_rows.contiguous()), _ffi.ptr(b_rows.contiguous()),
                                  _ffi.ptr(simplex.to(torch.float32).contiguous()), int(solver_iterations),
                                  _ffi.ptr(pen), _ffi.stream_ptr(a_rows.device)), "cotix_epa")
    return pen


# _contact_funcs registry (cotix/_colliders.py:21-35): (type, type) -> fn id
contact_funcs = {
    (AABB, AABB): _ffi.FN_AABB_AABB,
    (Circle, Circle): _ffi.FN_CIRCLE_CIRCLE,
    (Circle, AABB): _ffi.FN_CIRCLE_AABB,
    (Polygon, Polygon): _ffi.FN_POLY_POLY,
    (AABB, Polygon): _ffi.FN_AABB_POLY,
    (Circle, Polygon): _ffi.FN_CIRCLE_POLY,
    (Circle, Polygon4): _ffi.FN_CIRCLE_POLY,
    (Circle, Polygon6): _ffi.FN_CIRCLE_POLY,
    (AABB, Polygon4): _ffi.FN_AABB_POLY,
    (AABB, Polygon6): _ffi.FN_AABB_POLY,
    (Polygon4, Polygon4): _ffi.FN_POLY_POLY,
    (Polygon4, Polygon6): _ffi.FN_POLY_POLY,
    (Polygon6, Polygon6): _ffi.FN_POLY_POLY,
}


def resolve_collision(dyn1, par1, dyn2, par2, contact, params=None):
    """Batched resolve_collision: dyn [n, 6] updated in place, par [n, 4]
    (mass, inertia, elasticity, friction), contact [n, 4] (pen, cp); params:
    the Baumgarte constants (parallax_amd.Params, None: 0.3 / 0.01)."""
    n = dyn1.shape[0]
    for t in (dyn1, dyn2):
        if not t.is_contiguous():
            raise ValueError("dyn tensors must be contiguous")
    _ffi.check(_ffi.lib.cotix_resolve_ex(n, _ffi.ptr(dyn1), _ffi.ptr(par1.contiguous()), _ffi.ptr(dyn2),
                                         _ffi.ptr(par2.contiguous()), _ffi.ptr(contact.contiguous()),
                                         _params_ref(params), _ffi.stream_ptr(dyn1.device)), "cotix_resolve_ex")
    return dyn1, dyn2
