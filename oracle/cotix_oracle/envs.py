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
    """world.forward; a state (bodies, key, err) also carries the env's error
    bits (OR-ed, as the kernel's err word)."""
    from .geometry import ErrorFlag
    bodies, key = state[0], state[1]
    bodies = [copy.copy(b) for b in bodies]
    ef = None
    if len(state) > 2:
        ef = ErrorFlag()
        ef.bits = int(state[2])
    bodies, key = step(bodies, key, d0, ef, None, dt, action=dv, action_body=action_body)
    return (bodies, key) if ef is None else (bodies, key, ef.bits)


def eval_env(step, state, control, judge, eval_period, num_NFEs, WFE_scale, d0, action_body, carry=None):
    """-> (state, reward); with carry=(reward, finished) given, the loop starts
    from that carry and returns (state, reward, finished)."""
    tpn = F(eval_period / num_NFEs)
    dt = F(tpn / F(float(WFE_scale)))
    reward, finished = (F(0.0), False) if carry is None else (F(carry[0]), bool(carry[1]))
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
    return (state, reward) if carry is None else (state, reward, finished)


class LinearJudge:
    """Restatement of the device judge (include/cotix_amd.h cotix_judge,
    parallax_amd.envs.LinearJudge) over oracle states (bodies, key[, err]):
    state word k = body k // 6, word k % 6 of (px, py, vx, vy, angle,
    angular_velocity).  Sums over the nonzero weights in k order from the
    first term; a region holds the state when it is strictly inside every
    bound."""

    def __init__(self, rate_w=None, end_w=None, regions=(), done_on_error=False, rate_regions=()):
        self.rate_terms = sorted((int(k), F(w)) for k, w in dict(rate_w or {}).items() if F(w) != 0)
        self.end_terms = sorted((int(k), F(w)) for k, w in dict(end_w or {}).items() if F(w) != 0)
        self.regions = [(int(b), [F(v) for v in lo], [F(v) for v in hi], F(r)) for b, lo, hi, r in regions]
        self.done_on_error = bool(done_on_error)
        # the rate's pieces over non-terminal boxes (body, lo, hi, rate_w, bias): piecewise linear
        self.rate_regions = [(int(b), [F(v) for v in lo], [F(v) for v in hi],
                              sorted((int(k), F(w)) for k, w in dict(pw or {}).items() if F(w) != 0), F(pb))
                             for b, lo, hi, pw, pb in rate_regions]

    @staticmethod
    def _s(state, k):
        return F(state[0][k // 6].dyn()[k % 6])

    def _lin(self, state, terms):
        acc = None
        with np.errstate(all="ignore"):
            for k, w in terms:
                t = F(w * self._s(state, k))
                acc = t if acc is None else F(acc + t)
        return F(0.0) if acc is None else acc

    def region(self, state, boxes=None):
        for r, (b, lo, hi) in enumerate(x[:3] for x in (self.regions if boxes is None else boxes)):
            d = state[0][b].dyn()
            if all(bool(F(lo[q]) < F(d[q])) and bool(F(d[q]) < F(hi[q])) for q in range(6)):
                return r
        return -1

    def rate(self, state, sig):
        """base (+ the piece of the first rate region holding the state): each
        a sum from its first term; base + piece when both have terms"""
        acc = self._lin(state, self.rate_terms) if self.rate_terms else None
        r = self.region(state, self.rate_regions)
        if r >= 0:
            terms, b = self.rate_regions[r][3:]
            with np.errstate(all="ignore"):
                pc = self._lin(state, terms) if terms else None
                if b != 0:
                    pc = b if pc is None else F(pc + b)
                if pc is not None:
                    acc = pc if acc is None else F(acc + pc)
        return F(0.0) if acc is None else acc

    def is_done(self, state, sig):
        err = state[2] if len(state) > 2 else 0
        return self.region(state) >= 0 or (self.done_on_error and err != 0)

    def end_reward(self, state, sig):
        acc = self._lin(state, self.end_terms)
        r = self.region(state)
        if r >= 0:
            with np.errstate(all="ignore"):
                acc = F(acc + self.regions[r][3]) if self.end_terms else self.regions[r][3]
        return acc


class AffineControl:
    """Restatement of the device control (include/cotix_amd.h cotix_control):
    dv[i] = sum_q gain[i][q] * (target[i][q] - s[q]) (+ bias[i]) on `body`."""

    def __init__(self, body, gain=None, target=None, bias=(0.0, 0.0), clip=None):
        z = [[0.0] * 6, [0.0] * 6]
        self.body = int(body)
        self.gain = [[F(v) for v in row] for row in (gain or z)]
        self.target = [[F(v) for v in row] for row in (target or z)]
        self.bias = [F(v) for v in bias]
        self.clip = None if clip is None else [(F(lo), F(hi)) for lo, hi in clip]  # the saturating form

    def dv(self, state):
        s = state[0][self.body].dyn()
        out = []
        with np.errstate(all="ignore"):
            for i in range(2):
                acc = None
                for q in range(6):
                    if self.gain[i][q] != 0:
                        t = F(self.gain[i][q] * F(self.target[i][q] - F(s[q])))
                        acc = t if acc is None else F(acc + t)
                if self.bias[i] != 0:
                    acc = self.bias[i] if acc is None else F(acc + self.bias[i])
                acc = F(0.0) if acc is None else acc
                if self.clip is not None:  # jnp.clip (jax 0.4.x): minimum(hi, maximum(lo, x))
                    from .geometry import clip as _clip
                    lo, hi = self.clip[i]
                    acc = F(_clip(acc, lo, hi))
                out.append(acc)
        return tuple(out)

    def __call__(self, state):
        return self.dv, self


class HeldImpulse:
    """env.step(action): a constant dense signal (the held action)."""

    def __init__(self, dv):
        self.dv = (F(dv[0]), F(dv[1]))

    def __call__(self, state):
        return (lambda s: self.dv), self
