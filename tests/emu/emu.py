"""TEST INFRASTRUCTURE ONLY: ctypes front-end of the host emulation of the
fused step kernel (tests/emu/cotix_emu.cpp)."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
P_ = ctypes.c_void_p


def load(asan=False, path=None):
    """The host build (tests/emu/Makefile; __graft_entry__.build() builds the
    plain one), or the build at `path` (a variant).  Missing is an error, not a
    skip."""
    path = path or os.path.join(HERE, "build", "libcotix_emu_asan.so" if asan else "libcotix_emu.so")
    if not os.path.exists(path):
        raise FileNotFoundError("%s missing: run `make -C tests/emu` (or python __graft_entry__.py)" % path)
    lib = ctypes.CDLL(path)
    lib.emu_scene_create.argtypes = [ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, ctypes.POINTER(P_)]
    lib.emu_scene_create_ex.argtypes = [ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, P_, ctypes.POINTER(P_)]
    lib.emu_scene_create_ex2.argtypes = [ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, P_, ctypes.c_int,
                                         ctypes.POINTER(P_)]
    lib.emu_contacts_ex.argtypes = [ctypes.c_int, ctypes.c_int, P_, P_, P_, P_, P_]
    lib.emu_gjk.argtypes = [ctypes.c_int, P_, P_, P_, P_, P_]
    lib.emu_epa.argtypes = [ctypes.c_int, P_, P_, P_, ctypes.c_int, P_]
    lib.emu_step.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                             ctypes.c_int, P_, ctypes.c_int, P_, P_, ctypes.c_int]
    lib.emu_step_ex.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, P_, ctypes.c_int]
    lib.emu_contacts.argtypes = [ctypes.c_int, ctypes.c_int, P_, P_, P_, P_]
    lib.emu_order_clockwise.argtypes = [P_, ctypes.c_int, ctypes.c_int]
    lib.emu_gjk_start.argtypes = [ctypes.c_int, P_, P_, ctypes.c_int, P_]
    lib.emu_circle_poly_check.argtypes = [ctypes.c_int, P_, P_, P_, P_]
    lib.emu_body_penetration.argtypes = [P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P_, P_]
    lib.emu_body_aabb.argtypes = [P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, P_, P_]
    lib.emu_rollout.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, P_, P_, ctypes.c_int]
    lib.emu_rollout_backward.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_int, P_, ctypes.c_int, P_, P_, P_, ctypes.c_int]
    lib.emu_rollout_tape_words.argtypes = [P_]
    lib.emu_eval.argtypes = [P_, P_, P_, P_, P_, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_float, ctypes.c_int, P_, P_, P_, ctypes.c_int, P_, P_, ctypes.c_int, P_, P_, P_,
                             ctypes.c_int]
    lib.emu_last_error.restype = ctypes.c_char_p
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(P_)


TYPE_ID = {"Circle": 0, "AABB": 1, "Polygon": 2, "Polygon3": 3, "Polygon4": 4, "Polygon5": 5, "Polygon6": 6}


def params_ref(params):
    """An oracle Params (cotix_oracle.params) as a cotix_params pointer, or NULL."""
    return None if params is None else ctypes.cast(ctypes.pointer(params.c_struct()), P_)


def oracle_scene(lib, bodies, params=None, per_env_params=False):
    """Scene + local geometry from oracle Body objects; params: an oracle
    Params (cotix_oracle.params), None: the defaults.  per_env_params: the
    scene reads every env's body parameters from its geometry row, after the
    parts' words returned here (COTIX_SCENE_PER_ENV_BODY_PARAMS)."""
    prm = params
    bparams = np.array([[b.mass, b.inertia, b.elasticity, b.friction_coefficient] for b in bodies], np.float32)
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
    pb, pt, pn = (np.array(x, np.int32) for x in (pb, pt, pn))
    h = P_()
    cp = None if prm is None else prm.c_struct()
    rc = lib.emu_scene_create_ex2(len(bodies), _p(bparams), len(pb), _p(pb), _p(pt), _p(pn),
                                  None if cp is None else ctypes.cast(ctypes.pointer(cp), P_),
                                  1 if per_env_params else 0, ctypes.byref(h))
    if rc:
        raise RuntimeError(lib.emu_last_error().decode())
    return h, np.array(geom, np.float32)


def step(lib, h, dyn, keys, err, geom, gstride, n_steps, stages, dt=1e-2, E=16, dyn_reset=None, resets=None):
    """dyn f32 [nb, 6, B], keys u32 [B, 2], err u32 [B]: updated in place."""
    B = dyn.shape[2]
    for a in (dyn, keys, err, geom):
        assert a.flags.c_contiguous
    lib.emu_step(h, _p(dyn), _p(keys), _p(err), _p(geom), gstride, B, n_steps, dt, stages, None, 0,
                 _p(dyn_reset), _p(resets), E)


def step_ex(lib, h, dyn, keys, err, geom, gstride, n_steps, stages, nb, dt=1e-2, E=4, action=None, action_body=0,
            dyn_reset=None, resets=None):
    """step() with actions and the collider trace; returns (chosen i32
    [n_steps, nb, B], cells i32 [n_steps, nb, nb, B])."""
    B = dyn.shape[2]
    ch = np.full((n_steps, nb, B), -7, np.int32)
    cl = np.full((n_steps, nb, nb, B), -7, np.int32)
    act = None if action is None else np.ascontiguousarray(action, np.float32)
    lib.emu_step_ex(h, _p(dyn), _p(keys), _p(err), _p(geom), gstride, B, n_steps, dt, stages, _p(act), action_body,
                    _p(dyn_reset), _p(resets), _p(ch), _p(cl), E)
    return ch, cl


def rollout(lib, h, dyn, keys, err, geom, gstride, stages, actions, action_body, w, dt=1e-2, E=4):
    """Forward of the differentiable rollout; returns (ret [B], saved_dyn
    [T,ceil(B/4),nb*6,4], saved_keys [T,B,2], tape [T,ceil(B/4),tape_words,4]
    -- the library's env-block layout, cxk::row_at); dyn/keys/err advanced in
    place.  The tape is poisoned first (words the forward leaves unwritten are
    never read)."""
    T, B = actions.shape[0], dyn.shape[2]
    nblk = (B + 3) // 4
    ret = np.zeros(B, np.float32)
    sd = np.zeros((T, nblk, dyn.shape[0] * 6, 4), np.float32)
    sk = np.zeros((T, B, 2), np.uint32)
    tape = np.full((T, nblk, lib.emu_rollout_tape_words(h), 4), 0x7FBADBAD, np.uint32)
    actions = np.ascontiguousarray(actions, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    lib.emu_rollout(h, _p(dyn), _p(keys), _p(err), _p(geom), gstride, B, T, dt, stages, _p(actions), action_body,
                    _p(w), _p(ret), _p(sd), _p(sk), _p(tape), E)
    return ret, sd, sk, tape


def rollout_backward(lib, h, sd, sk, geom, gstride, stages, actions, action_body, w, dt=1e-2, E=4, tape=None):
    """The backward: from the forward's tape (MODE 4), or re-playing the
    forward (tape None, MODE 2)."""
    T, B = actions.shape[0], actions.shape[1]
    ga = np.zeros((T, B, 2), np.float32)
    gd = np.zeros((sd.shape[2] // 6, 6, B), np.float32)
    actions = np.ascontiguousarray(actions, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    rc = lib.emu_rollout_backward(h, _p(sd), _p(sk), _p(tape), _p(geom), gstride, B, T, dt, stages, _p(actions),
                                  action_body, _p(w), _p(ga), _p(gd), E)
    if rc:
        raise RuntimeError(lib.emu_last_error().decode())
    return ga, gd


def eval_(lib, h, dyn, keys, err, geom, gstride, n_nfe, wfe, dt, stages, judge=None, control=None, action=None,
          action_body=0, reward=None, finished=None, reset_mode=0, dyn_reset=None, resets=None, obs=None, E=4):
    """cotix_eval on the host (numpy arrays updated in place; judge / control
    are ctypes cotix_judge / cotix_control structs or None)."""
    ref = lambda s: None if s is None else ctypes.cast(ctypes.pointer(s), P_)  # noqa: E731
    rc = lib.emu_eval(h, _p(dyn), _p(keys), _p(err), _p(geom), gstride, dyn.shape[2], n_nfe, wfe, dt, stages,
                      ref(judge), ref(control), _p(action), action_body, _p(reward), _p(finished), reset_mode,
                      _p(dyn_reset), _p(resets), _p(obs), E)
    if rc:
        raise RuntimeError(lib.emu_last_error().decode())
