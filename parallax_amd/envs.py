"""The reference's continuous-time environment API (cotix/_envs.py:9-132,
cotix/_controls.py:6-27), batched over envs, over the fused step kernel.

AbstractEnvironment.eval(eval_period, num_NFEs, WFE_scale) follows the
reference loop exactly (cotix/_envs.py:37-132): per NFE the control yields a
dense control function; the world is advanced WFE_scale times by
dt = time_per_NFE / WFE_scale, the judge's reward rate is integrated
(reward += judge(s, u) * dt), and an env whose judge says is_done is frozen at
that point with its end reward -- here per env, with torch.where over the
batch.  The reference ships no concrete AbstractWorld (SimpleWorld is broken,
SURVEY.md §2); PhysicsWorld is the build's: one launch of the fused step per
forward, the control signal entering through the kernel's velocity-impulse
hook (added after Euler, where the LunarLander driver adds gravity).

State, rewards and flags are device tensors with the env batch as the last
(state) or only (reward, flags) dimension; judges and controls are torch code.
"""
import numpy as np
import torch

from . import _ffi


class WorldState:
    """dyn f32 [n_bodies][6][B], keys i32 [B][2], err i32 [B] (device)."""

    def __init__(self, dyn, keys, err):
        self.dyn, self.keys, self.err = dyn, keys, err

    def clone(self):
        return WorldState(self.dyn.clone(), self.keys.clone(), self.err.clone())

    @staticmethod
    def where(mask, a, b):
        """Per env: a where mask[env] else b."""
        return WorldState(torch.where(mask, a.dyn, b.dyn), torch.where(mask[:, None], a.keys, b.keys),
                          torch.where(mask, a.err, b.err))


class AbstractControlSignal:
    """cotix/_controls.py:6-15: a dense control signal evaluated on a state."""

    def apply(self, state, dt):
        raise NotImplementedError


class VelocityImpulse(AbstractControlSignal):
    """Δv [B, 2] added to the velocity of `body` right after Euler (the
    kernel's action hook; config-5 convention)."""

    def __init__(self, dv, body):
        self.dv, self.body = dv, body

    def apply(self, state, dt):
        return self.dv


class AbstractControl:
    """cotix/_controls.py:18-27: __call__(state) -> (dense_fn, new_control),
    dense_fn(state) -> AbstractControlSignal."""

    def __call__(self, state):
        raise NotImplementedError

    def select(self, mask, other):
        """Per-env choice between two control states (frozen envs keep theirs).
        Stateless controls need not override this."""
        return self


class AbstractJudge:
    """cotix/_envs.py:9-32: reward rate, is_done, end_reward -- each [B]."""

    def __call__(self, state, control_signal):
        raise NotImplementedError

    def is_done(self, state, control_signal):
        raise NotImplementedError

    def end_reward(self, state, control_signal):
        raise NotImplementedError


class AbstractWorld:
    def forward(self, state, control_signal, dt):
        raise NotImplementedError


class PhysicsWorld(AbstractWorld):
    """forward = one fused driver step (Euler -> [impulse] -> collider ->
    constraints -> key split) of the given World's scene."""

    def __init__(self, world, stages=_ffi.STAGES_ROBOCUP):
        self.world, self.stages = world, stages

    def forward(self, state, control_signal, dt):
        out = state.clone()
        action, body = None, 0
        if control_signal is not None:
            action = control_signal.apply(state, dt)[None]
            body = control_signal.body
        self.world.step_state(out.dyn, out.keys, out.err, 1, dt, self.stages, action, body)
        return out


class AbstractEnvironment:
    """world, state, control, judge as in cotix/_envs.py:35-41."""

    def __init__(self, world, state, control, judge):
        self.world, self.state, self.control, self.judge = world, state, control, judge

    def eval(self, eval_period, num_NFEs, WFE_scale=10):
        """-> (new environment with the end state, reward [B]); the reference's
        cotix/_envs.py:37-132, per env."""
        B = self.state.err.shape[0]
        dev = self.state.err.device
        tpn = float(np.float32(eval_period / num_NFEs))  # the carry's f32 time_per_NFE
        dt = float(np.float32(np.float32(tpn) / np.float32(float(WFE_scale))))
        state, control = self.state, self.control
        reward = torch.zeros(B, dtype=torch.float32, device=dev)
        finished = torch.zeros(B, dtype=torch.bool, device=dev)
        for _ in range(num_NFEs):
            dense_fn, new_control = control(state)
            new_state = state
            signal = dense_fn(new_state)
            end_reward = torch.where(finished, reward, reward + self.judge.end_reward(new_state, signal))
            pre_state, pre_control, pre_reward = state, control, end_reward  # possible premature out
            already = self.judge.is_done(new_state, signal).to(torch.bool)
            for _ in range(WFE_scale):
                new_state = self.world.forward(new_state, signal, dt)
                signal = dense_fn(new_state)
                ending_reward = reward + self.judge.end_reward(new_state, signal)
                now = self.judge.is_done(new_state, signal).to(torch.bool) & ~already
                pre_state = WorldState.where(now, new_state, pre_state)
                pre_control = new_control.select(now, pre_control)
                pre_reward = torch.where(now, ending_reward, pre_reward)
                already = already | now
                reward = reward + self.judge(new_state, signal) * dt
            state = WorldState.where(already, pre_state, new_state)
            control = pre_control.select(already, new_control)
            reward = torch.where(already, pre_reward, reward)
            finished = already
        out = AbstractEnvironment(self.world, state, self.control, self.judge)
        return out, reward
