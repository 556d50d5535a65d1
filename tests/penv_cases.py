"""Per-env body parameters (include/cotix_amd.h COTIX_SCENE_PER_ENV_BODY_PARAMS):
a vmapped LunarLander (cotix/_lunar_lander.py:29-143) whose terrain AND whose
lander / leg mass, inertia, elasticity and friction_coefficient vary per env
(domain randomization over the parameter leaves, cotix/_bodies.py:140-154),
started with the legs on the landing pad so that GJK/EPA contacts, the
resolutions (which read every parameter) and the joints act from the first
step.  Test infrastructure (CPU emulation and GPU tests)."""
import numpy as np

from cotix_oracle import physics as P
from cotix_oracle import prng

F = np.float32


def lunar_penv_bodies(B, seed=0):
    """Per env the oracle bodies (randomized parameters, per-env terrain)."""
    rng = np.random.default_rng(seed)
    keys = [np.asarray(k, np.uint32) for k in prng.split(prng.PRNGKey(31 + seed), B)]
    out = []
    for e in range(B):
        ob = P.lunar_lander_bodies(keys[e])
        lander, rleg, lleg, _ = ob
        lander.mass, lander.inertia = F(rng.uniform(10.0, 60.0)), F(rng.uniform(10.0, 60.0))
        lander.elasticity, lander.friction_coefficient = F(rng.uniform(0.2, 1.0)), F(rng.uniform(0.02, 0.6))
        for leg in (rleg, lleg):
            leg.mass, leg.inertia = F(rng.uniform(0.3, 3.0)), F(rng.uniform(0.3, 3.0))
            leg.elasticity, leg.friction_coefficient = F(rng.uniform(0.2, 1.0)), F(rng.uniform(0.02, 0.6))
        dx, dy = rng.uniform(-0.3, 0.3), -(5.0 + 1.2) - 0.02 + rng.uniform(-0.05, 0.05)
        for b in (lander, rleg, lleg):
            b.position = (F(b.position[0] + dx), F(b.position[1] + dy))
            b.velocity = (F(rng.uniform(-0.5, 0.5)), F(rng.uniform(-1.0, 0.2)))
            b.angular_velocity = F(rng.uniform(-0.5, 0.5))
        out.append(ob)
    return out


def rows(cport_scene_of, obs):
    """Per-env geometry rows [B, G]: the env's parts (the C port's layout)
    followed by its [n_bodies][4] parameters."""
    r = []
    for ob in obs:
        g = cport_scene_of(ob)
        par = np.array([[b.mass, b.inertia, b.elasticity, b.friction_coefficient] for b in ob], F).reshape(-1)
        r.append(np.concatenate([g, par]))
    return np.ascontiguousarray(np.stack(r), F)


def state(obs):
    """dyn f32 [nb, 6, B] and collider keys u32 [B, 2]."""
    dyn = np.ascontiguousarray(np.stack([np.array([b.dyn() for b in ob], F) for ob in obs], axis=2))
    keys = np.ascontiguousarray(np.asarray(prng.split(prng.PRNGKey(5), len(obs)), np.uint32))
    return dyn, keys
