"""Random multi-part bodies for the body-level operator tests."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, "golden"), os.path.join(HERE, "..", "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import make_golden as mg  # noqa: E402
from cotix_oracle import geometry as G  # noqa: E402
from cotix_oracle import physics as P  # noqa: E402

F = np.float32


def bodies(seed=0):
    rng = np.random.default_rng(seed)
    b0 = P.Body([G.Circle(F(0.4), (F(0.3), F(0.0))), G.AABB((F(-0.5), F(-0.2)), (F(0.2), F(0.4)))], mass=1.0)
    b1 = P.Body([mg.rand_poly(rng, 4), G.Circle(F(0.25), (F(-0.4), F(0.1)))], mass=1.0)
    b2 = P.Body([mg.rand_poly(rng, 6), G.AABB((F(0.1), F(-0.6)), (F(0.7), F(0.0)))], mass=1.0)
    return [b0, b1, b2]


def states(B, seed=1):
    """dyn [3, 6, B]: bodies scattered around the origin, random angles."""
    rng = np.random.default_rng(seed)
    dyn = np.zeros((3, 6, B), np.float32)
    for b in range(3):
        dyn[b, 0] = rng.uniform(-1.0, 1.0, B)
        dyn[b, 1] = rng.uniform(-1.0, 1.0, B)
        dyn[b, 4] = rng.uniform(-3.2, 3.2, B)
    dyn[1, :2, ::7] = dyn[0, :2, ::7]  # some coincident centres
    return np.ascontiguousarray(dyn)


def oracle_body(make, dyn, e, b):
    body = make()[b]
    body.set_dyn(dyn[b, :, e])
    return body
