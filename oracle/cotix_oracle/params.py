"""TEST INFRASTRUCTURE ONLY -- CPU oracle, never imported by the product path.

The reference's hard-coded constants on the hot path as one parameter block
(include/cotix_amd.h ``cotix_params``), defaults = the reference's literals:

  prng_layout       "legacy"  jax_threefry_partitionable=False (JAX 0.4.x default)
                              or "partitionable" (the default from JAX 0.5); the
                              reference pins no JAX version (pyproject.toml:16)
  baumgarte         0.3       cotix/_collision_resolution.py:105
  baumgarte_dt      0.01      cotix/_collision_resolution.py:115
  contact_p         0.5       cotix/_colliders.py:220-223
  gjk_max_steps     32        cotix/_collisions.py:101
  epa_max_iters     48        cotix/_contacts.py:271,295 (the min(48, ...) cap)
  epa_circle_iters  128       cotix/_contacts.py:162-163
  epa_body_iters    48        cotix/_universal_shape.py:120

The oracle reads the block in force (``current()``); ``use(p)`` scopes one.
"""
import contextlib
import ctypes
from dataclasses import dataclass

LAYOUTS = {"legacy": 0, "partitionable": 1}


@dataclass(frozen=True)
class Params:
    prng_layout: str = "legacy"
    baumgarte: float = 0.3
    baumgarte_dt: float = 0.01
    contact_p: float = 0.5
    gjk_max_steps: int = 32
    epa_max_iters: int = 48
    epa_circle_iters: int = 128
    epa_body_iters: int = 48

    @property
    def partitionable(self):
        return self.prng_layout == "partitionable"

    def c_struct(self):
        """struct cotix_params (also the C port's OParams: same field order)."""
        return CParams(LAYOUTS[self.prng_layout], self.baumgarte, self.baumgarte_dt, self.contact_p,
                       self.gjk_max_steps, self.epa_max_iters, self.epa_circle_iters, self.epa_body_iters)


class CParams(ctypes.Structure):
    _fields_ = [("prng_layout", ctypes.c_int), ("baumgarte", ctypes.c_float), ("baumgarte_dt", ctypes.c_float),
                ("contact_p", ctypes.c_float), ("gjk_max_steps", ctypes.c_int), ("epa_max_iters", ctypes.c_int),
                ("epa_circle_iters", ctypes.c_int), ("epa_body_iters", ctypes.c_int)]


DEFAULT = Params()
_stack = [DEFAULT]


def current():
    return _stack[-1]


@contextlib.contextmanager
def use(p):
    """Run the oracle with parameter block ``p`` (None: the defaults)."""
    _stack.append(DEFAULT if p is None else p)
    try:
        yield _stack[-1]
    finally:
        _stack.pop()
