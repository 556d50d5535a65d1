"""parallax_amd -- MI355X-native batched 2-D rigid-body stepper for cotix
(DelftMercurians/Parallax).  The hot path is HIP for gfx950 in
libcotix_amd.so (include/cotix_amd.h); this package is the Python host side
mirroring the reference's body/shape/operator surface.
"""
from . import _ffi  # noqa: F401  (raises ImportError when the HIP library is missing)
from . import random  # noqa: F401
from . import contracts, pytree, render  # noqa: F401
from .bodies import AnyBody, BodyView  # noqa: F401
from .env import BatchedEnv, StepResult  # noqa: F401
from .envs import (AbstractEnvironment, AffineControl, LinearJudge, PhysicsWorld, VelocityImpulse,  # noqa: F401
                   WorldState)
from .params import Params  # noqa: F401
from .physics import (ContactInfo, ExplicitEulerPhysics, RandomizedCollider, SimpleConstraintSolver,  # noqa: F401
                      check_for_collision_convex, compute_penetration_vector_convex, contact_funcs,
                      resolve_collision, run_contacts)
from .rollout import rollout as differentiable_rollout  # noqa: F401
from .rollout import rollout_backward, rollout_forward, trajectory  # noqa: F401
from .scenarios import BoxWorld, LunarLander, RoboCupEnv  # noqa: F401
from .shapes import AABB, Circle, Polygon, Polygon3, Polygon4, Polygon5, Polygon6, UniversalShape  # noqa: F401
from .world import Scene, World  # noqa: F401

__version__ = "0.2.0"
