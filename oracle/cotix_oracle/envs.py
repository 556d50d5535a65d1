"""TEST INFRASTRUCTURE ONLY -- single-env restatement of the reference's
continuous-time evaluation loop AbstractEnvironment.eval (cotix/_envs.py:37-132)
over the oracle step, with plain-Python control/judge callables.

control(state) -> (dense_fn, new_control); dense_fn(state) -> dv (f32[2], the
velocity impulse applied after Euler to `action_body`); judge has
rate(state, dv), is_done(state, dv), end_reward(state, dv).  `state` is
(bodies, key)."""
import copy

import numpy as np

F = np.float32


def _forward(step, state, dv, dt, d0, action_body):
    bodies, key = state
    bodies = [copy.copy(b) for b in bodies]
    bodies, key = step(bodies, key, d0, None, None, dt, action=dv, action_body=action_body)
    return (bodies, key)


def eval_env(step, state, control, judge, eval_period, num_NFEs, WFE_scale, d0, action_body):
    tpn = F(eval_period / num_NFEs)
    dt = F(tpn / F(float(WFE_scale)))
    reward = F(0.0)
    finished = False
    for _ in range(num_NFEs):
        dense_fn, new_control = control(state)
        new_state = state
        sig = dense_fn(new_state)
        end_reward = reward if finished else F(reward + judge.end_reward(new_state, sig))
        premature = (state, control, end_reward)
        already = bool(judge.is_done(new_state, sig))
        for _ in range(WFE_scale):
            new_state = _forward(step, new_state, sig, dt, d0, action_body)
            sig = dense_fn(new_state)
            ending_reward = F(reward + judge.end_reward(new_state, sig))
            if bool(judge.is_done(new_state, sig)) and not already:
                premature = (new_state, new_control, ending_reward)
                already = True
            reward = F(reward + F(judge.rate(new_state, sig)) * dt)
        if already:
            state, control, reward = premature
        else:
            state, control = new_state, new_control
        finished = already
    return state, reward
