"""Body descriptions (cotix/_bodies.py:135-186 AnyBody, :189-273 DynamicBody).

An AnyBody here describes one body of a batched world: its static
parameters (mass, inertia, elasticity, friction_coefficient: one value per
body, or a [B] tensor when they vary over the env batch -- a vmapped pytree,
e.g. domain randomization; the scene then carries them per env,
COTIX_SCENE_PER_ENV_BODY_PARAMS) and its initial dynamic state (position,
velocity, angle, angular_velocity: a value shared by all envs or a tensor with
a leading batch dimension).  Once placed in a World the live state is the
world's SoA tensor; ``World.body(i)`` returns a view.
"""
import torch

from .shapes import UniversalShape

DYN_FIELDS = ("px", "py", "vx", "vy", "angle", "angular_velocity")


def _param(x, name):
    """One value per body (a float) or one per env (a float32 [B] tensor)."""
    t = torch.as_tensor(x, dtype=torch.float32)
    if t.numel() == 1 and t.dim() <= 1:
        return float(t.reshape(()))
    if t.dim() != 1:
        raise ValueError("%s must be one value per body or a [B] tensor (one per env)" % name)
    return t.detach().to("cpu").contiguous()


class AnyBody:
    def __init__(self, mass=1.0, inertia=1.0, position=(0.0, 0.0), velocity=(0.0, 0.0), angle=0.0,
                 angular_velocity=0.0, elasticity=1.0, friction_coefficient=1.0, is_area=False, shape=None):
        if shape is None or not isinstance(shape, UniversalShape):
            raise TypeError("AnyBody needs a UniversalShape")
        self.mass = _param(mass, "mass")
        self.inertia = _param(inertia, "inertia")
        self.elasticity = _param(elasticity, "elasticity")
        self.friction_coefficient = _param(friction_coefficient, "friction_coefficient")
        self.position = torch.as_tensor(position, dtype=torch.float32)
        self.velocity = torch.as_tensor(velocity, dtype=torch.float32)
        self.angle = torch.as_tensor(angle, dtype=torch.float32)
        self.angular_velocity = torch.as_tensor(angular_velocity, dtype=torch.float32)
        self.is_area = is_area
        self.shape = shape

    def params(self):
        return [self.mass, self.inertia, self.elasticity, self.friction_coefficient]

    def params_per_env(self):
        """Whether some parameter is a [B] tensor (one value per env)."""
        return any(isinstance(v, torch.Tensor) for v in self.params())

    def param_columns(self, B):
        """[4, B] (mass, inertia, elasticity, friction) per env."""
        cols = []
        for v in self.params():
            t = torch.as_tensor(v, dtype=torch.float32)
            if t.dim() == 1 and t.shape[0] != B:
                raise ValueError("a per-env body parameter has %d envs, the world %d" % (t.shape[0], B))
            cols.append(t.expand(B))
        return torch.stack(cols, 0)

    def template_params(self):
        """The parameters as floats (env 0 of per-env ones): the scene's table."""
        return [float(v[0]) if isinstance(v, torch.Tensor) else v for v in self.params()]

    def dyn_columns(self, B):
        """[6, B] initial dynamic state."""
        p = self.position.expand(B, 2) if self.position.dim() == 1 else self.position
        v = self.velocity.expand(B, 2) if self.velocity.dim() == 1 else self.velocity
        a = self.angle.expand(B)
        w = self.angular_velocity.expand(B)
        return torch.stack([p[:, 0], p[:, 1], v[:, 0], v[:, 1], a, w], dim=0)


class BodyView:
    """Live view of body i of a World (AoS access with the reference's field
    names over the SoA device tensor)."""

    def __init__(self, world, i):
        self._w, self._i = world, i
        self.mass, self.inertia, self.elasticity, self.friction_coefficient = world.bodies[i].params()
        self.shape = world.bodies[i].shape

    @property
    def position(self):
        return self._w.dyn[self._i, 0:2].T

    @property
    def velocity(self):
        return self._w.dyn[self._i, 2:4].T

    @property
    def angle(self):
        return self._w.dyn[self._i, 4]

    @property
    def angular_velocity(self):
        return self._w.dyn[self._i, 5]
