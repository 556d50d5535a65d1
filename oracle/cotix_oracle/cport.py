"""TEST INFRASTRUCTURE ONLY -- ctypes front-end of the C port of the oracle
(oracle/c/cotix_oracle.c, built by `make -C oracle`).  Used by the tests as
a fast checker and by bench.py as the timed CPU baseline ("kind": "port")."""
import ctypes
import os
import time

import numpy as np

from . import physics as P
from . import prng

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "..", "build", "libcotix_oracle.so")
_P = ctypes.c_void_p
TYPE_ID = {"Circle": 0, "AABB": 1, "Polygon": 2, "Polygon3": 3, "Polygon4": 4, "Polygon5": 5, "Polygon6": 6}
STAGES_ROBOCUP = 1 | 4 | 16
STAGES_LUNAR = 1 | 2 | 4 | 8 | 16


def load():
    lib = ctypes.CDLL(LIB)
    lib.oracle_scene_size.restype = ctypes.c_int
    lib.oracle_scene_init.argtypes = [_P, ctypes.c_int, _P, ctypes.c_int, _P, _P, _P]
    lib.oracle_step.argtypes = [_P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                ctypes.c_int, _P, _P, ctypes.c_int]
    lib.oracle_step_ex.argtypes = [_P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                   ctypes.c_int, _P, ctypes.c_int, _P, _P, _P, _P, ctypes.c_int]
    lib.oracle_contacts.argtypes = [ctypes.c_int, ctypes.c_int, _P, _P, _P, _P]
    lib.oracle_contacts_ex.argtypes = [ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P]
    lib.oracle_scene_set_params.argtypes = [_P, _P]
    lib.oracle_scene_set_per_env_params.argtypes = [_P, ctypes.c_int]
    lib.oracle_gjk.argtypes = [ctypes.c_int, _P, _P, _P, _P, _P]
    lib.oracle_epa.argtypes = [ctypes.c_int, _P, _P, _P, ctypes.c_int, _P]
    lib.oracle_rollout.argtypes = [_P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                   ctypes.c_int, _P, ctypes.c_int, _P, _P, ctypes.c_int]
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_P)


def params_ref(params):
    """An oracle Params (cotix_oracle.params) as a pointer to the C port's
    OParams (the cotix_params layout), or NULL (the defaults)."""
    return None if params is None else ctypes.cast(ctypes.pointer(params.c_struct()), _P)


class Scene:
    """Scene description + local geometry (row) from oracle Body objects;
    params: an oracle Params (None: the reference's literals)."""

    def __init__(self, lib, bodies, params=None):
        self.lib = lib
        prm = params
        params = np.array([[b.mass, b.inertia, b.elasticity, b.friction_coefficient] for b in bodies], np.float32)
        pb, pt, pn, geom = [], [], [], []
        for i, b in enumerate(bodies):
            for p in b.parts:
                pb.append(i)
                pt.append(TYPE_ID[p.kind])
                if p.kind == "Circle":
                    pn.append(0)
                    geom += [p.radius, p.position[0], p.position[1], 0.0]
                elif p.kind == "AABB":
                    pn.append(0)
                    geom += [p.lower[0], p.lower[1], p.upper[0], p.upper[1]]
                else:
                    pn.append(len(p.vertices_))
                    for v in p.vertices_:
                        geom += [v[0], v[1]]
        self.n_bodies = len(bodies)
        self.geom = np.array(geom, np.float32)
        self.mem = ctypes.create_string_buffer(lib.oracle_scene_size())
        args = [np.array(x, np.int32) for x in (pb, pt, pn)]
        rc = lib.oracle_scene_init(self.mem, len(bodies), _p(params), len(pb), *[_p(a) for a in args])
        if rc:
            raise RuntimeError("oracle_scene_init failed (%d)" % rc)
        if prm is not None:
            cp = prm.c_struct()
            lib.oracle_scene_set_params(self.mem, ctypes.cast(ctypes.pointer(cp), _P))

    def set_per_env_params(self, on=True):
        """Every env's own (mass, inertia, elasticity, friction) per body, as
        [n_bodies * 4] floats after its part geometry in the per-env geometry
        rows (include/cotix_amd.h COTIX_SCENE_PER_ENV_BODY_PARAMS); returns the
        floats per row."""
        return self.lib.oracle_scene_set_per_env_params(self.mem, 1 if on else 0)

    def step(self, dyn, keys, err, n_steps, stages, geom=None, dyn_reset=None, resets=None, nthreads=0, dt=1e-2):
        """dyn f32 [nb,6,B], keys u32 [B,2], err u32 [B] (in place); geom None
        (shared, this scene's) or f32 [B,G] per env."""
        B = dyn.shape[2]
        g = self.geom if geom is None else np.ascontiguousarray(geom, np.float32)
        gstride = 0 if geom is None else g.shape[1]
        self.lib.oracle_step(self.mem, _p(dyn), _p(keys), _p(err), _p(g), gstride, B, n_steps, dt, stages,
                             _p(dyn_reset), _p(resets), nthreads)

    def step_ex(self, dyn, keys, err, n_steps, stages, geom=None, action=None, action_body=0, dyn_reset=None,
                resets=None, trace=False, nthreads=0, dt=1e-2):
        """step() with actions [n_steps, B, 2] and the collider trace: returns
        (chosen i32 [n_steps, nb, B], cells i32 [n_steps, nb, nb, B]) or None."""
        B = dyn.shape[2]
        g = self.geom if geom is None else np.ascontiguousarray(geom, np.float32)
        gstride = 0 if geom is None else g.shape[1]
        ch = cl = None
        if trace:
            ch = np.full((n_steps, self.n_bodies, B), -7, np.int32)
            cl = np.full((n_steps, self.n_bodies, self.n_bodies, B), -7, np.int32)
        act = None if action is None else np.ascontiguousarray(action, np.float32)
        self.lib.oracle_step_ex(self.mem, _p(dyn), _p(keys), _p(err), _p(g), gstride, B, n_steps, dt, stages,
                                _p(act), action_body, _p(dyn_reset), _p(resets), _p(ch), _p(cl), nthreads)
        return (ch, cl) if trace else None

    def rollout(self, dyn, keys, err, stages, actions, action_body, ret_w, geom=None, nthreads=0, dt=1e-2):
        """Forward of the differentiable rollout; returns ret [B]."""
        B = dyn.shape[2]
        g = self.geom if geom is None else np.ascontiguousarray(geom, np.float32)
        gstride = 0 if geom is None else g.shape[1]
        ret = np.zeros(B, np.float32)
        actions = np.ascontiguousarray(actions, np.float32)
        ret_w = np.ascontiguousarray(ret_w, np.float32)
        self.lib.oracle_rollout(self.mem, _p(dyn), _p(keys), _p(err), _p(g), gstride, B, actions.shape[0], dt, stages,
                                _p(actions), action_body, _p(ret_w), _p(ret), nthreads)
        return ret


def fd_action_grad(sc, dyn0, keys0, actions, action_body, ret_w, stages, eps=1e-3, nthreads=0):
    """Central finite differences d ret / d action [T, B, 2] of the C port:
    4T perturbed rollouts per env, batched (OpenMP over all of them)."""
    nb, _, B = dyn0.shape
    T = actions.shape[0]
    n = 4 * T
    dyn = np.ascontiguousarray(np.repeat(dyn0[:, :, None, :], n, axis=2).reshape(nb, 6, n * B))
    keys = np.ascontiguousarray(np.repeat(keys0[None], n, axis=0).reshape(n * B, 2))
    acts = np.repeat(actions[:, None], n, axis=1).copy()  # [T, n, B, 2]
    for q in range(n):
        t, c, sgn = q // 4, (q // 2) % 2, 1.0 if q % 2 == 0 else -1.0
        acts[t, q, :, c] += np.float32(sgn * eps)
    acts = np.ascontiguousarray(acts.reshape(T, n * B, 2))
    err = np.zeros(n * B, np.uint32)
    ret = sc.rollout(dyn, keys, err, stages, acts, action_body, ret_w, nthreads=nthreads).reshape(n, B)
    g = (ret[0::2].astype(np.float64) - ret[1::2]) / (2 * eps)  # [2T, B]
    return g.reshape(T, 2, B).transpose(0, 2, 1)


def robocup_batch(B, seed_keys=3, offset=0, total=None):
    """The bench's RoboCup batch for global env ids offset .. offset+B-1 of a
    `total`-env run (perturbed ball per env from split(PRNGKey(2), total),
    keys split(PRNGKey(3), total); global env 0 unperturbed)."""
    from . import geometry  # noqa: F401
    total = B if total is None else total
    keys = np.ascontiguousarray(prng.split(prng.PRNGKey(seed_keys), total)[offset:offset + B]).astype(np.uint32)
    base = np.array([b.dyn() for b in P.robocup_bodies()], np.float32)
    dyn = np.repeat(base[:, :, None], B, axis=2)
    pk = prng.split(prng.PRNGKey(2), total)
    for e in range(B):
        if offset + e == 0:
            continue
        kp, kv, kw = prng.split(pk[offset + e], 3)
        u = prng.uniform(kp, (2,))
        lo, hi = np.array([-4.4, -2.9], np.float32), np.array([4.4, 2.9], np.float32)
        pos = np.maximum(lo, u * (hi - lo) + lo)
        vel = prng.uniform(kv, (2,), -2.0, 2.0)
        w = prng.uniform(kw, (), -10.0, 10.0)
        dyn[4, :, e] = [pos[0], pos[1], vel[0], vel[1], 0.0, w]
    return np.ascontiguousarray(dyn), keys


def time_baseline(scenario, seconds=12.0, B=1024):
    """Env-steps/s of the C port on this host's cores (OpenMP over envs),
    over a bounded sample of the bench workload (autoreset, 4 steps/call)."""
    lib = load()
    nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    if scenario == "robocup":
        sc = Scene(lib, P.robocup_bodies())
        dyn, keys = robocup_batch(B)
        geom, stages = None, STAGES_ROBOCUP
    else:
        tk = prng.split(prng.PRNGKey(0), B)
        sc = Scene(lib, P.lunar_lander_bodies(tk[0]))
        rows = [Scene(lib, P.lunar_lander_bodies(k)).geom for k in tk]
        geom = np.ascontiguousarray(np.stack(rows))
        dyn = np.ascontiguousarray(np.repeat(np.array([b.dyn() for b in P.lunar_lander_bodies(tk[0])],
                                                      np.float32)[:, :, None], B, axis=2))
        keys = np.ascontiguousarray(prng.split(prng.PRNGKey(1), B)).astype(np.uint32)
        stages = STAGES_LUNAR
    reset = dyn.copy()
    err = np.zeros(B, np.uint32)
    resets = np.zeros(B, np.uint32)
    n = 0
    sc.step(dyn, keys, err, 1, stages, geom, reset, resets, nthreads)  # warm-up
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        sc.step(dyn, keys, err, 4, stages, geom, reset, resets, nthreads)
        n += 4 * B
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env-steps/s", "cores": nthreads, "kind": "port",
            "sample": "%d env-steps (%d envs x %d steps, %s, autoreset) of the C oracle port "
                      "(faithful N1xN2 collider scan), OpenMP %d threads, %.1f s"
                      % (n, B, n // B, scenario, nthreads, dt)}
