"""The reference's two scenarios, batched.

RoboCupEnv   cotix/_robocup.py:9-130     (5 bodies, AABB + Circle parts)
LunarLander  cotix/_lunar_lander.py:26-218 (4 bodies, Polygon4/Polygon6 parts)

Constants are built with the same float32 operations the JAX constructors
perform (numpy float32 scalar arithmetic on the host: construction data, not
the hot path).  The only constants that need a transcendental -- the rotated
leg quads of LunarLander (cos/sin(-0.3), cotix/_lunar_lander.py:44-72) --
are given as the float32 bit patterns the build's deterministic sin/cos
produce (tests/test_scenarios_cpu.py re-derives them with the oracle).
Per-env randomness (terrain, perturbations) is drawn on the device with the
HIP threefry kernels.
"""
import numpy as np
import torch

from . import _ffi
from . import random as jr
from .bodies import AnyBody
from .shapes import AABB, Circle, Polygon4, Polygon6, UniversalShape
from .world import World

F = np.float32
INF = float("inf")


def env_range(batch, env_offset, total_envs):
    """Validated global env range of a (shard) batch: returns total_envs.
    Every slice of a global key split goes through here, so a shard outside
    the global batch is an error, not a short key tensor."""
    batch, env_offset = int(batch), int(env_offset)
    total = batch if total_envs is None else int(total_envs)
    if batch < 0 or env_offset < 0 or env_offset + batch > total:
        raise ValueError("env range [%d, %d) outside the global batch of %d envs"
                         % (env_offset, env_offset + batch, total))
    return total


# ---------------------------------------------------------------------------
# RoboCup
# ---------------------------------------------------------------------------
def robocup_bodies():
    """RoboCupEnv.__init__ (cotix/_robocup.py:14-130)."""
    f2 = F(2)
    fd = (F(10.4), F(7.4))
    field = AABB([-fd[0] / f2, -fd[1] / f2], [fd[0] / f2, fd[1] / f2])
    play_lo = (F(-9) / f2, F(-6) / f2)
    play = AABB(list(play_lo), [F(9) / f2, F(6) / f2])
    gd0, gd1, gw = F(0.2), F(1.0), F(0.01)
    yb_lo = (play_lo[0] - gd0, F(-0.5))
    yb_up = (play_lo[0], F(0.5))
    ya = ((yb_lo[0], yb_lo[1]), (yb_lo[0] + gw, yb_lo[1] + gd1))
    yb = ((yb_lo[0] - (-gw), yb_lo[1] - F(0)), (yb_lo[0] + gd0, yb_lo[1] + gw))
    yc = ((yb_up[0] - gd0, yb_up[1] - gw), yb_up)

    def aabb(lu):
        return AABB([lu[0][0], lu[0][1]], [lu[1][0], lu[1][1]])

    def refl(lu):  # reflect_aabb_by_y_axis :63-69
        return AABB([-lu[1][0], lu[0][1]], [-lu[0][0], lu[1][1]])

    ball_r = F(0.022) * F(3)
    return [
        AnyBody(shape=UniversalShape(field), mass=INF, is_area=True),
        AnyBody(shape=UniversalShape(play), mass=INF, is_area=True),
        AnyBody(shape=UniversalShape(aabb(ya), aabb(yb), aabb(yc)), mass=INF, elasticity=0.5),
        AnyBody(shape=UniversalShape(refl(ya), refl(yb), refl(yc)), mass=INF, elasticity=0.5),
        AnyBody(shape=UniversalShape(Circle(ball_r, [0.0, 0.0])), mass=0.5, position=[0.0, 0.0],
                velocity=[1.0, 0.01], angular_velocity=10.0, elasticity=1.0),
    ]


def robocup_perturbation(B, seed=2, device="cuda", offset=0, total=None, layout=None):
    """The build's batched-reset scheme for the envs
    with GLOBAL ids offset .. offset+B-1 of a `total`-env batch (default: B,
    offset 0), so a rank's shard equals the same envs of one big run: global
    env 0 is the exact reference state; env g >= 1 gets, from
    split(PRNGKey(seed), total)[g] -> (kp, kv, kw) = split(., 3): ball position
    U([-4.4,4.4] x [-2.9,2.9]), velocity U([-2,2]^2), angular velocity
    U(-10,10).  Returns the ball's [6, B] dynamic columns.  layout: the PRNG
    layout of every draw (parallax_amd.random)."""
    total = env_range(B, offset, total)
    k = jr.split(jr.PRNGKey(seed, device), total, layout)[offset:offset + B].contiguous()
    kk = jr.split(k, 3, layout)
    u = jr.uniform(kk[:, 0], 2, layout=layout)
    lo = torch.tensor([-4.4, -2.9], dtype=torch.float32, device=device)
    hi = torch.tensor([4.4, 2.9], dtype=torch.float32, device=device)
    pos = torch.maximum(lo, u * (hi - lo) + lo)
    vel = jr.uniform(kk[:, 1], 2, -2.0, 2.0, layout)
    w = jr.uniform(kk[:, 2], None, -10.0, 10.0, layout)
    cols = torch.stack([pos[:, 0], pos[:, 1], vel[:, 0], vel[:, 1], torch.zeros_like(w), w], 0)
    if offset == 0 and B > 0:
        cols[:, 0] = torch.tensor([0.0, 0.0, 1.0, 0.01, 0.0, 10.0], dtype=torch.float32, device=device)
    return cols


class RoboCupEnv:
    """RoboCupEnv with a batch dimension.  ``keys``: collider keys [B, 2]
    (default split(PRNGKey(3), total)[offset:offset+B]); ``perturb``: apply
    robocup_perturbation.  ``env_offset`` / ``total_envs``: this batch holds the
    envs with global ids env_offset .. env_offset+B-1 of a total_envs-env run
    (a rank's shard); defaults: 0 and B.  ``params``: the scene's
    parameter block (parallax_amd.Params; its PRNG layout also draws the keys
    and perturbations)."""

    stages = _ffi.STAGES_ROBOCUP

    def __init__(self, batch=1, device="cuda", keys=None, perturb=False, perturb_seed=2, env_offset=0,
                 total_envs=None, params=None):
        self.bodies = robocup_bodies()
        total = env_range(batch, env_offset, total_envs)
        if keys is None:
            keys = jr.split(jr.PRNGKey(3, device), total, params)[env_offset:env_offset + batch].contiguous()
        self.world = World(self.bodies, batch, device, keys, params)
        if perturb:
            self.world.dyn[4] = robocup_perturbation(batch, perturb_seed, device, env_offset, total, params)
        self.dyn_reset = self.world.dyn.clone()

    # field green, goals yellow / blue, ball red; white field outlines, no
    # outline pass for the ball (cotix/_robocup.py:131-138)
    colors = [(0, 180, 0)] * 2 + [(255, 255, 0), (0, 128, 255), (255, 0, 0)]
    edge_colors = [(255, 255, 255)] * 2 + [(255, 255, 0), (0, 128, 255), None]

    def draw(self, painter, env=0, prims=None):
        """RoboCupEnv.draw(painter) (cotix/_robocup.py:140-150) for one env:
        the geometry comes from the device render kernel."""
        from . import render as R
        cmds = R.commands_bodies(self.bodies, self.colors, self.edge_colors)
        R.replay(painter, cmds, R.render(self.world) if prims is None else prims, env)


# ---------------------------------------------------------------------------
# BoxWorld: a generic finite-dynamics scene (NOT a reference scenario)
# ---------------------------------------------------------------------------
def box_world_bodies():
    """Balls in an open box, built from the reference's own body/shape API
    (AnyBody, UniversalShape, AABB, Circle): 3 static non-overlapping walls
    (floor, left, right; elasticity 0.8, friction 0.3) and 4 balls of finite
    mass and inertia.  Unlike RoboCup (whose overlapping static bodies drive
    every env to NaN within two steps) every contact here has
    finite operands, so it times the full-cost contact/resolution path.  The
    ball parameters are env 0 of tests/golden/make_golden.box_world_bodies."""
    walls = [AABB([-3.0, -3.2], [3.0, -2.0]), AABB([-4.0, -1.9], [-3.0, 3.0]), AABB([3.0, -1.9], [4.0, 3.0])]
    bodies = [AnyBody(shape=UniversalShape(w), mass=INF, elasticity=0.8, friction_coefficient=0.3) for w in walls]
    rng = np.random.default_rng(100)
    for _ in range(4):
        rng.uniform(size=4)  # (position, velocity: drawn per env on the device instead)
        r, m, i = F(rng.uniform(0.3, 0.7)), F(rng.uniform(0.5, 2.0)), F(rng.uniform(0.2, 1.0))
        rng.uniform(-5, 5)
        e, f = F(rng.uniform(0.3, 1.0)), F(rng.uniform(0.1, 0.9))
        bodies.append(AnyBody(shape=UniversalShape(Circle(r, [0.0, 0.0])), mass=float(m), inertia=float(i),
                              elasticity=float(e), friction_coefficient=float(f)))
    return bodies


class BoxWorld:
    """BoxWorld with a batch dimension: per env (global ids env_offset ..
    env_offset+B-1 of total_envs) the 4 balls start at uniform positions in
    [-2.8, 2.8] x [-1.5, 2.5], velocities U(-3, 3)^2 and spins U(-5, 5) drawn
    from split(PRNGKey(seed), total)[id]; collider keys split(PRNGKey(seed+1),
    total)[id].  Driver stages as RoboCup (Euler -> collider -> key split).
    ``params``: the scene's parameter block (its PRNG layout draws the keys too)."""

    stages = _ffi.STAGES_ROBOCUP

    def __init__(self, batch=1, device="cuda", seed=9, env_offset=0, total_envs=None, params=None):
        self.bodies = box_world_bodies()
        total = env_range(batch, env_offset, total_envs)
        sl = slice(env_offset, env_offset + batch)
        keys = jr.split(jr.PRNGKey(seed + 1, device), total, params)[sl].contiguous()
        self.world = World(self.bodies, batch, device, keys, params)
        kb = jr.split(jr.split(jr.PRNGKey(seed, device), total, params)[sl].contiguous(), 4, params)  # [B, 4, 2]
        for k in range(4):
            u = jr.uniform(kb[:, k].contiguous(), 5, layout=params)
            d = self.world.dyn[3 + k]
            d[0] = u[:, 0] * 5.6 - 2.8
            d[1] = u[:, 1] * 4.0 - 1.5
            d[2] = u[:, 2] * 6.0 - 3.0
            d[3] = u[:, 3] * 6.0 - 3.0
            d[4] = 0.0
            d[5] = u[:, 4] * 10.0 - 5.0
        self.dyn_reset = self.world.dyn.clone()


# ---------------------------------------------------------------------------
# LunarLander
# ---------------------------------------------------------------------------
LANDER_POLY = [(-14, 17), (-17, 0), (-17, -10), (17, -10), (17, 0), (14, 17)]
LEG_AWAY, LEG_DOWN = 24, 8


def _bits(*hx):
    return np.array(hx, dtype=np.uint32).view(np.float32)


# left leg after sort -> rotate(-0.3) -> *0.05 (cotix/_lunar_lander.py:32-66)
LEFT_LEG = _bits(0x3CB9BFBD, 0xBED2C897, 0x3E5ADF1D, 0xBEB485B4, 0xBCB9BFBD, 0x3ED2C897, 0xBE5ADF1D,
                 0x3EB485B4).reshape(4, 2)
RIGHT_LEG = LEFT_LEG * np.array([-1.0, 1.0], dtype=np.float32)  # :68-72 (not re-sorted)


def lunar_terrain(keys, layout=None):
    """cotix/_lunar_lander.py:109-132 per env: keys [B, 2] -> quads [B, 7, 4, 2]
    (unsorted; Polygon4 sorts them when the world uploads geometry)."""
    ks = jr.split(keys, 5, layout)
    h = jr.uniform(ks[:, 0], 8, -5.0, 5.0, layout).clone()
    h[:, 0] = h[:, 0] * 10.0
    h[:, 3] = -2.0
    h[:, 4] = -2.0
    h[:, 7] = h[:, 7] * 10.0
    B = keys.shape[0]
    dev = keys.device
    pos = torch.empty(B, 8, dtype=torch.float32, device=dev)
    pos[:, 0] = -100.0
    pos[:, 1] = jr.uniform(ks[:, 1], None, -12.0, -9.0, layout)
    pos[:, 2] = jr.uniform(ks[:, 2], None, -8.0, -4.0, layout)
    pos[:, 3] = -2.0
    pos[:, 4] = 2.0
    pos[:, 5] = jr.uniform(ks[:, 3], None, 4.0, 8.0, layout)
    pos[:, 6] = jr.uniform(ks[:, 4], None, 9.0, 12.0, layout)
    pos[:, 7] = 100.0
    m10 = torch.full((B, 7), -10.0, device=dev)
    p1 = torch.stack([pos[:, :7], h[:, :7]], -1)
    p2 = torch.stack([pos[:, :7], m10], -1)
    p3 = torch.stack([pos[:, 1:], h[:, 1:]], -1)
    p4 = torch.stack([pos[:, 1:], m10], -1)
    return torch.stack([p1, p2, p3, p4], 2)


def lunar_lander_bodies(terrain):
    """LunarLander.__init__ (cotix/_lunar_lander.py:29-143); terrain [B, 7, 4, 2]."""
    f05 = F(0.05)
    lander_v = [[F(x) * f05, F(y) * f05] for x, y in LANDER_POLY]
    center = (F(0.0), F(5.0))
    lleg = [F(LEG_AWAY) * f05 + center[0], F(-LEG_DOWN) * f05 + center[1]]
    rleg = [F(-LEG_AWAY) * f05 + center[0], F(-LEG_DOWN) * f05 + center[1]]
    lander = AnyBody(shape=UniversalShape(Polygon6(lander_v)), position=list(center), mass=30.0, inertia=30.0,
                     angle=0.01, friction_coefficient=0.1)
    right_leg = AnyBody(shape=UniversalShape(Polygon4(RIGHT_LEG, presorted=True)), position=rleg, inertia=1.0,
                        friction_coefficient=0.1)
    left_leg = AnyBody(shape=UniversalShape(Polygon4(LEFT_LEG, presorted=True)), position=lleg, inertia=1.0,
                       friction_coefficient=0.1)
    ground = AnyBody(shape=UniversalShape(*[Polygon4(terrain[:, k].cpu()) for k in range(7)]), mass=INF,
                     inertia=INF, elasticity=0.1, friction_coefficient=0.1)
    return [lander, right_leg, left_leg, ground]


class LunarLander:
    """LunarLander with a batch dimension.  ``key``: terrain key(s) -- one
    key [2] (every env the same terrain) or [B, 2]; default PRNGKey(0).
    ``collider_keys`` default split(PRNGKey(1), B) (env 0 of a batch of 1:
    PRNGKey(0), the reference's examples/test_viz.py:46).  ``params``: the
    scene's parameter block (its PRNG layout also draws the terrain)."""

    stages = _ffi.STAGES_LUNAR

    def __init__(self, key=None, batch=1, device="cuda", collider_keys=None, params=None):
        if key is None:
            key = jr.PRNGKey(0, device)
        key = key.to(device)
        keys = key.expand(batch, 2).contiguous() if key.dim() == 1 else key
        terrain = lunar_terrain(keys, params)
        self.bodies = lunar_lander_bodies(terrain)
        if collider_keys is None:
            collider_keys = (jr.PRNGKey(0, device)[None] if batch == 1
                             else jr.split(jr.PRNGKey(1, device), batch, params))
        self.world = World(self.bodies, batch, device, collider_keys, params)
        self.dyn_reset = self.world.dyn.clone()
        # the polygon broadphase (results unchanged: the kernel certifies every pair it skips)
        self.stages = _ffi.STAGES_LUNAR | _ffi.STAGE_BROADPHASE

    def step(self):
        """LunarLander.step(): the joint constraints (cotix/_lunar_lander.py:145-218)."""
        self.world.lunar_constraints()
        return self

    def draw(self, painter, env=0, prims=None):
        """LunarLander.draw(painter) (cotix/_lunar_lander.py:220-225) for one
        env: every body with the shapes' default colours, then the two red
        landing-zone lines."""
        from . import render as R
        red = (255, 0, 0)
        cmds = R.commands_bodies(self.bodies, extra_lines=[((-2, -1.8), (-2, -1.0), red), ((2, -1.8), (2, -1.0), red)])
        R.replay(painter, cmds, R.render(self.world) if prims is None else prims, env)
