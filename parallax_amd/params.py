"""The reference's hard-coded hot-path constants as one parameter block
(include/cotix_amd.h ``cotix_params``), given to a scene at creation.

  prng_layout       "legacy"   every jax.random call of the step: JAX's
                               jax_threefry_partitionable=False layout (the
                               0.4.x default) or "partitionable" (the default
                               from JAX 0.5); the reference pins no JAX
                               version (pyproject.toml:16)
  baumgarte         0.3        cotix/_collision_resolution.py:105
  baumgarte_dt      0.01       cotix/_collision_resolution.py:115 ("/ dt is missing")
  contact_p         0.5        cotix/_colliders.py:220-223 (a candidate's bernoulli)
  gjk_max_steps     32         cotix/_collisions.py:101
  epa_max_iters     48         cotix/_contacts.py:271,295 (the min(48, ...) cap)
  epa_circle_iters  128        cotix/_contacts.py:162-163
  epa_body_iters    48         cotix/_universal_shape.py:120
"""
import ctypes
from dataclasses import dataclass

import numpy as np

LAYOUTS = {"legacy": 0, "partitionable": 1}


class CotixParams(ctypes.Structure):
    """struct cotix_params (include/cotix_amd.h)."""
    _fields_ = [("prng_layout", ctypes.c_int), ("baumgarte", ctypes.c_float), ("baumgarte_dt", ctypes.c_float),
                ("contact_p", ctypes.c_float), ("gjk_max_steps", ctypes.c_int), ("epa_max_iters", ctypes.c_int),
                ("epa_circle_iters", ctypes.c_int), ("epa_body_iters", ctypes.c_int)]


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

    def __post_init__(self):
        if self.prng_layout not in LAYOUTS:
            raise ValueError("prng_layout must be one of %s" % sorted(LAYOUTS))
        # the block holds float32 values, as the kernels do (a block read back
        # from the library compares equal to the one it was made from)
        for f in ("baumgarte", "baumgarte_dt", "contact_p"):
            object.__setattr__(self, f, float(np.float32(getattr(self, f))))

    @property
    def layout_id(self):
        return LAYOUTS[self.prng_layout]

    def c_struct(self):
        return CotixParams(self.layout_id, self.baumgarte, self.baumgarte_dt, self.contact_p, self.gjk_max_steps,
                           self.epa_max_iters, self.epa_circle_iters, self.epa_body_iters)

    @classmethod
    def from_c(cls, c):
        inv = {v: k for k, v in LAYOUTS.items()}
        return cls(inv[c.prng_layout], c.baumgarte, c.baumgarte_dt, c.contact_p, c.gjk_max_steps, c.epa_max_iters,
                   c.epa_circle_iters, c.epa_body_iters)


DEFAULT = Params()


def layout_id(layout):
    """A layout name ("legacy" / "partitionable"), a Params, or None (legacy) -> COTIX_PRNG_*."""
    if layout is None:
        return 0
    if isinstance(layout, Params):
        return layout.layout_id
    if layout not in LAYOUTS:
        raise ValueError("unknown PRNG layout %r" % (layout,))
    return LAYOUTS[layout]
