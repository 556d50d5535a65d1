"""Shared control/judge pairs for the AbstractEnvironment.eval tests: a torch
version (batched, product side) and a numpy version (single env, oracle side)
with the same f32 operations, so results compare bit for bit."""
import numpy as np
import torch

from parallax_amd import envs as E

F = np.float32
K, VT, XT = 0.05, (1.0, 0.0), 1.2


class PDControl(E.AbstractControl):
    """dv = K * (VT - v_body): a stateless dense control."""

    def __init__(self, body):
        self.body = body

    def __call__(self, state):
        def dense(s):
            v = s.dyn[self.body, 2:4, :].T  # [B, 2]
            vt = torch.tensor(VT, dtype=torch.float32, device=v.device)
            return E.VelocityImpulse((K * (vt - v)).contiguous(), self.body)
        return dense, self


class XJudge(E.AbstractJudge):
    """rate = x_body; done when x_body > XT; end reward = 2 * y_body."""

    def __init__(self, body):
        self.body = body

    def __call__(self, state, sig):
        return state.dyn[self.body, 0, :]

    def is_done(self, state, sig):
        return state.dyn[self.body, 0, :] > XT

    def end_reward(self, state, sig):
        return 2.0 * state.dyn[self.body, 1, :]


class OraclePD:
    def __init__(self, body):
        self.body = body

    def __call__(self, state):
        def dense(s):
            v = s[0][self.body].velocity
            return (F(K) * (F(VT[0]) - v[0]), F(K) * (F(VT[1]) - v[1]))
        return dense, self


class OracleX:
    def __init__(self, body):
        self.body = body

    def rate(self, state, sig):
        return state[0][self.body].position[0]

    def is_done(self, state, sig):
        return state[0][self.body].position[0] > F(XT)

    def end_reward(self, state, sig):
        return F(2.0) * state[0][self.body].position[1]
