"""Differentiable fused rollout (BASELINE config 5): grad(return)/d(action)
through an n-step rollout, forward and backward as HIP kernels
(cotix_rollout_ex / cotix_rollout_backward_ex, include/cotix_amd.h).  The
forward writes a decision tape (each step's resolutions and, for polygon
contacts, EPA's final edge) and the backward restores those decisions instead
of re-playing the collider; tape=False runs the re-play instead (the same
bits, the check of the tape path).

The reference defines neither action nor return (cotix/_envs.py:9-28 is
abstract); SURVEY.md 8(d) fixes them: action[t] (f32[B,2]) is added to the
velocity of `action_body` right after Euler -- where the LunarLander driver
adds gravity (examples/test_viz.py:27-31) -- and the return is
    R[env] = sum_{t=1..T} sum_k w[k] * state_t[k]      (terms with w[k] == 0 skipped)
over the n_bodies*6 state words (default: the ball's x position, body 4 of
RoboCup).  Derivatives are jax.grad's through the reference: the executed
branch of every lax.cond, RandomizedCollider choices held fixed, balanced
ties for max/min/clip.  Circle, AABB and polygon contacts (GJK/EPA through
EPA's final edge and contact_from_edges), circle x polygon contacts (through
every GJK / EPA point the circle's direction-dependent support builds) and
the LunarLander joints (stages=_ffi.STAGES_LUNAR).
"""
import numpy as np
import torch

from . import _ffi


def ball_x_weights(n_bodies, body=4, coord=0):
    w = np.zeros(n_bodies * 6, np.float32)
    w[body * 6 + coord] = 1.0
    return w


def _weights(world, w):
    nb = len(world.bodies)
    w = ball_x_weights(nb, nb - 1) if w is None else np.ascontiguousarray(np.asarray(w, np.float32).reshape(-1))
    if w.shape != (nb * 6,):
        raise ValueError("return weights must have n_bodies*6 entries")
    return w


def _check_actions(world, actions):
    actions = actions.to(world.device, torch.float32).contiguous()
    if actions.dim() != 3 or actions.shape[1:] != (world.B, 2):
        raise ValueError("actions must be [T, B, 2]")
    return actions


def rollout_forward(world, actions, action_body=None, ret_weights=None, dt=1e-2, stages=_ffi.STAGES_ROBOCUP,
                    tape=True):
    """Run T = actions.shape[0] fused steps (world state advanced in place)
    and save the trajectory (and the decision tape).  Returns (ret [B],
    saved) for rollout_backward.

    Memory: the saved trajectory is T * (24 * n_bodies + 8) bytes per env;
    the decision tape adds T * tape_words * 4 bytes per env, where
    tape_words = cotix_rollout_tape_words(scene) is 12 * n_bodies in analytic
    scenes (RoboCup: 60 words = 240 B per env-step, twice the saved state)
    and 5 * n_bodies + 4 * n_contacts in polygon scenes (it grows with the
    distinct contact count).  tape=False skips it: the backward then re-plays
    the collider (same bits, slower); an allocation failure of the tape says
    so."""
    actions = _check_actions(world, actions)
    nb, B, T = len(world.bodies), world.B, actions.shape[0]
    action_body = nb - 1 if action_body is None else int(action_body)
    w = _weights(world, ret_weights)
    nblk = (B + 3) // 4  # the saved rows in env blocks of 4 (include/cotix_amd.h, trajectory())
    saved_dyn = torch.empty(T, nblk, nb * 6, 4, device=world.device, dtype=torch.float32)
    saved_keys = torch.empty(T, B, 2, device=world.device, dtype=torch.int32)
    tw = _ffi.lib.cotix_rollout_tape_words(world.scene.handle)
    try:
        tp = torch.empty(T, nblk, tw, 4, device=world.device, dtype=torch.int32) if tape else None
    except torch.OutOfMemoryError as e:
        raise torch.OutOfMemoryError(
            "rollout decision tape: %d x %d x %d u32 words (%.1f MiB) do not fit; tape=False runs the re-play "
            "backward without it (%s)" % (T, tw, B, T * tw * B * 4 / 2**20, e)) from e
    ret = torch.zeros(B, device=world.device, dtype=torch.float32)
    _ffi.check(_ffi.lib.cotix_rollout_ex(
        world.scene.handle, _ffi.ptr(world.dyn), _ffi.ptr(world.keys), _ffi.ptr(world.err), _ffi.ptr(world.geom),
        world.geom_stride, B, T, float(dt), int(stages), _ffi.ptr(actions), action_body,
        w.ctypes.data_as(_ffi._P), _ffi.ptr(ret), _ffi.ptr(saved_dyn), _ffi.ptr(saved_keys), _ffi.ptr(tp),
        _ffi.stream_ptr(world.device)), "cotix_rollout_ex")
    saved = dict(dyn=saved_dyn, keys=saved_keys, tape=tp, actions=actions, action_body=action_body, w=w,
                 dt=float(dt), stages=int(stages))
    return ret, saved


def trajectory(saved, B):
    """The saved states before each step as [T, n_bodies, 6, B] (a copy): the
    library keeps them in env blocks of 4, [T][ceil(B/4)][n_bodies*6][4], so
    that a wave of 4 envs saves and restores one contiguous run."""
    sd = saved["dyn"]
    T, nblk, nd, _ = sd.shape
    return sd.permute(0, 2, 1, 3).reshape(T, nd // 6, 6, nblk * 4)[..., :B].contiguous()


def rollout_backward(world, saved, want_dyn0=False, replay=False):
    """d ret / d actions [T, B, 2] (and d ret / d initial state [nb, 6, B]):
    from the forward's tape, or (replay=True, or no tape saved) re-playing
    the forward's steps."""
    nb, B = len(world.bodies), world.B
    T = saved["actions"].shape[0]
    ga = torch.empty(T, B, 2, device=world.device, dtype=torch.float32)
    gd = torch.empty(nb, 6, B, device=world.device, dtype=torch.float32) if want_dyn0 else None
    tp = None if replay else saved.get("tape")
    _ffi.check(_ffi.lib.cotix_rollout_backward_ex(
        world.scene.handle, _ffi.ptr(saved["dyn"]), _ffi.ptr(saved["keys"]), _ffi.ptr(tp), _ffi.ptr(world.geom),
        world.geom_stride, B, T, saved["dt"], saved["stages"], _ffi.ptr(saved["actions"]), saved["action_body"],
        saved["w"].ctypes.data_as(_ffi._P), _ffi.ptr(ga), _ffi.ptr(gd), _ffi.stream_ptr(world.device)),
        "cotix_rollout_backward_ex")
    return ga, gd


class _Rollout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, actions, world, action_body, ret_weights, dt, stages):
        ret, saved = rollout_forward(world, actions.detach(), action_body, ret_weights, dt, stages)
        ctx.world, ctx.saved = world, saved
        return ret

    @staticmethod
    def backward(ctx, g_ret):
        ga, _ = rollout_backward(ctx.world, ctx.saved)
        return ga * g_ret.to(ga.dtype)[None, :, None], None, None, None, None, None


def rollout(world, actions, action_body=None, ret_weights=None, dt=1e-2, stages=_ffi.STAGES_ROBOCUP):
    """R[env] (differentiable w.r.t. actions via torch.autograd); advances
    `world` by T steps in place."""
    return _Rollout.apply(actions, world, action_body, ret_weights, dt, stages)
