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


def _f32(x):
    return float(np.float32(x))


def _tuples(x):
    return tuple(_tuples(v) for v in x) if isinstance(x, (list, tuple)) else x


class _Frozen:
    """Immutable after construction (nested lists become tuples): a prepared
    launch copies the device struct once (BatchedEnv._launcher), so an
    in-place change could never reach the kernel -- it raises instead."""

    def _freeze(self):
        for k, v in vars(self).items():
            object.__setattr__(self, k, _tuples(v))
        object.__setattr__(self, "_frozen", True)

    def __setattr__(self, name, value):
        if getattr(self, "_frozen", False):
            raise AttributeError("%s is immutable: build a new one" % type(self).__name__)
        object.__setattr__(self, name, value)


class LinearJudge(_Frozen, AbstractJudge):
    """A device AbstractJudge (include/cotix_amd.h cotix_judge): over the env's
    state words s[k] (k = 6 * body + {px, py, vx, vy, angle, angular_velocity})

      judge(s)      = sum_k rate_w[k] * s[k]  (+ piece_r(s) in rate region r: piecewise linear)
      end_reward(s) = sum_k end_w[k] * s[k] (+ the reward of the first region holding s)
      is_done(s)    = some region holds s, or (done_on_error and err bits set)

    sums over the nonzero weights in k order, from the first term.
    regions: [(body, lo[6], hi[6], reward)], strictly inside every bound
    (NaN never inside, +-inf leaves a word free); at most 4, and at most 16
    nonzero weights per sum.  rate_regions: [(body, lo[6], hi[6], rate_w,
    bias)], boxes held like the regions but not terminal: while rate region r
    is the first holding s, the reward rate gains piece_r(s) = sum_k w[k] *
    s[k] (+ bias) (at most 8 nonzero weights, at most 4 rate regions); the
    rate is base + piece when both have terms.  The torch methods evaluate the
    same f32 expressions in the same order as the kernel, so the host loop and
    the fused cotix_eval agree bit for bit."""

    def __init__(self, rate_w=None, end_w=None, regions=(), done_on_error=False, rate_regions=()):
        self.rate = sorted((int(k), _f32(w)) for k, w in dict(rate_w or {}).items() if _f32(w) != 0.0)
        self.end = sorted((int(k), _f32(w)) for k, w in dict(end_w or {}).items() if _f32(w) != 0.0)
        self.regions = [(int(b), [_f32(v) for v in lo], [_f32(v) for v in hi], _f32(r)) for b, lo, hi, r in regions]
        self.done_on_error = bool(done_on_error)
        self.rate_regions = [(int(b), [_f32(v) for v in lo], [_f32(v) for v in hi],
                              sorted((int(k), _f32(w)) for k, w in dict(pw or {}).items() if _f32(w) != 0.0),
                              _f32(pb)) for b, lo, hi, pw, pb in rate_regions]
        if len(self.rate) > 16 or len(self.end) > 16 or len(self.regions) > _ffi.JUDGE_REGIONS:
            raise ValueError("LinearJudge: at most 16 nonzero weights per sum and 4 regions")
        if len(self.rate_regions) > _ffi.JUDGE_REGIONS or any(len(t) > 8 for *_, t, _ in self.rate_regions):
            raise ValueError("LinearJudge: at most 4 rate regions of at most 8 nonzero weights")
        if any(len(lo) != 6 or len(hi) != 6 for _, lo, hi, *_ in self.regions + self.rate_regions):
            raise ValueError("LinearJudge: region bounds are 6 words (one body's state)")
        self._freeze()

    def c_struct(self):
        j = _ffi.CotixJudge()
        for k, w in self.rate:
            j.rate_w[k] = w
        for k, w in self.end:
            j.end_w[k] = w
        j.n_regions = len(self.regions)
        for r, (b, lo, hi, rew) in enumerate(self.regions):
            j.region_body[r] = b
            for q in range(6):
                j.region_lo[r][q] = lo[q]
                j.region_hi[r][q] = hi[q]
            j.region_reward[r] = rew
        j.done_on_error = int(self.done_on_error)
        j.n_rate_regions = len(self.rate_regions)
        for r, (body, lo, hi, terms, b) in enumerate(self.rate_regions):
            j.rate_region_body[r] = body
            for q in range(6):
                j.rate_region_lo[r][q] = lo[q]
                j.rate_region_hi[r][q] = hi[q]
            for k, w in terms:
                j.rate_region_w[r][k] = w
            j.rate_region_bias[r] = b
        return j

    @staticmethod
    def _word(state, k):
        return state.dyn[k // 6, k % 6, :]

    def _lin(self, state, terms):
        acc = None
        for k, w in terms:
            t = self._word(state, k) * torch.tensor(w, dtype=torch.float32, device=state.dyn.device)
            acc = t if acc is None else acc + t
        return torch.zeros_like(state.dyn[0, 0, :]) if acc is None else acc

    def _region(self, state, boxes=None):
        """index of the first region (or box of `boxes`) holding the state, -1
        for none ([B] int)."""
        boxes = self.regions if boxes is None else boxes
        B = state.dyn.shape[2]
        r_of = torch.full((B,), -1, dtype=torch.int64, device=state.dyn.device)
        for r in reversed(range(len(boxes))):
            b, lo, hi = boxes[r][:3]
            inside = torch.ones(B, dtype=torch.bool, device=state.dyn.device)
            for q in range(6):
                v = state.dyn[b, q, :]
                inside = inside & (torch.tensor(lo[q], dtype=torch.float32, device=v.device) < v) & \
                    (v < torch.tensor(hi[q], dtype=torch.float32, device=v.device))
            r_of = torch.where(inside, torch.full_like(r_of, r), r_of)
        return r_of

    def __call__(self, state, control_signal):
        acc = None if not self.rate else self._lin(state, self.rate)
        if not self.rate_regions:
            return self._lin(state, self.rate)
        r_of = self._region(state, self.rate_regions)
        out = torch.zeros_like(state.dyn[0, 0, :]) if acc is None else acc
        for r, (_, _, _, terms, b) in enumerate(self.rate_regions):
            if not terms and b == 0.0:
                continue
            pc = None if not terms else self._lin(state, terms)
            if b != 0.0:
                bt = torch.tensor(b, dtype=torch.float32, device=out.device)
                pc = bt.expand_as(out) if pc is None else pc + bt
            out = torch.where(r_of == r, pc if acc is None else acc + pc, out)
        return out

    def is_done(self, state, control_signal):
        d = self._region(state) >= 0
        if self.done_on_error:
            d = d | (state.err != 0)
        return d

    def end_reward(self, state, control_signal):
        acc = self._lin(state, self.end)
        r_of = self._region(state)
        for r, (_, _, _, rew) in enumerate(self.regions):
            rt = torch.tensor(rew, dtype=torch.float32, device=acc.device)
            acc = torch.where(r_of == r, acc + rt if self.end else rt.expand_as(acc), acc)
        return acc


class AffineControl(_Frozen, AbstractControl):
    """A device AbstractControl (include/cotix_amd.h cotix_control): the dense
    signal is the velocity impulse dv[i] = sum_q gain[i][q] * (target[i][q] -
    s[q]) (+ bias[i]) on `body`, from that body's state s before each
    env-step (nonzero gains in q order from the first term, bias last when
    nonzero).  clip = ((lo0, hi0), (lo1, hi1)): the saturating form dv[i] =
    clip(dv[i], lo_i, hi_i) (jnp.clip: NaN propagates).  Stateless."""

    def __init__(self, body, gain=None, target=None, bias=(0.0, 0.0), clip=None):
        self.body = int(body)
        z = [[0.0] * 6, [0.0] * 6]
        self.gain = [[_f32(v) for v in row] for row in (gain or z)]
        self.target = [[_f32(v) for v in row] for row in (target or z)]
        self.bias = [_f32(v) for v in bias]
        self.clip = None if clip is None else [(_f32(lo), _f32(hi)) for lo, hi in clip]
        if self.clip is not None and (len(self.clip) != 2 or any(np.isnan(v) for p in self.clip for v in p)):
            raise ValueError("AffineControl: clip is ((lo0, hi0), (lo1, hi1)), no NaN bound")
        self._freeze()

    def c_struct(self):
        c = _ffi.CotixControl()
        c.body = self.body
        for i in range(2):
            for q in range(6):
                c.gain[i][q] = self.gain[i][q]
                c.target[i][q] = self.target[i][q]
            c.bias[i] = self.bias[i]
        if self.clip is not None:
            c.saturate = 1
            for i in range(2):
                c.clip_lo[i], c.clip_hi[i] = self.clip[i]
        return c

    def dv(self, state):
        out = []
        for i in range(2):
            acc = None
            for q in range(6):
                g = self.gain[i][q]
                if g != 0.0:
                    v = state.dyn[self.body, q, :]
                    tg = torch.tensor(self.target[i][q], dtype=torch.float32, device=v.device)
                    t = torch.tensor(g, dtype=torch.float32, device=v.device) * (tg - v)
                    acc = t if acc is None else acc + t
            if self.bias[i] != 0.0:
                bt = torch.tensor(self.bias[i], dtype=torch.float32, device=state.dyn.device)
                acc = bt.expand(state.dyn.shape[2]).clone() if acc is None else acc + bt
            acc = torch.zeros_like(state.dyn[0, 0, :]) if acc is None else acc
            if self.clip is not None:  # jnp.clip = min(hi, max(lo, x)): ties keep the bound, NaN propagates
                lo, hi = (torch.tensor(v, dtype=torch.float32, device=acc.device) for v in self.clip[i])
                acc = torch.where(lo >= acc, lo, acc)
                acc = torch.where(hi <= acc, hi, acc)
            out.append(acc)
        return torch.stack(out, 1).contiguous()

    def __call__(self, state):
        return (lambda s: VelocityImpulse(self.dv(s), self.body)), self


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

    def fused(self):
        """True when eval runs as ONE cotix_eval launch: a PhysicsWorld with a
        device judge (LinearJudge) and a device control (AffineControl or None)."""
        return (isinstance(self.world, PhysicsWorld) and isinstance(self.judge, LinearJudge)
                and (self.control is None or isinstance(self.control, AffineControl)))

    def eval(self, eval_period, num_NFEs, WFE_scale=10, fused=None):
        """-> (new environment with the end state, reward [B]); the reference's
        cotix/_envs.py:37-132, per env.  With a device judge and control
        (fused(), or fused=True) the whole NFE x WFE loop is one kernel launch
        (cotix_eval); otherwise the loop runs here, one launch per env-step."""
        B = self.state.err.shape[0]
        dev = self.state.err.device
        tpn = float(np.float32(eval_period / num_NFEs))  # the carry's f32 time_per_NFE
        dt = float(np.float32(np.float32(tpn) / np.float32(float(WFE_scale))))
        if self.fused() if fused is None else fused:
            return self._eval_fused(num_NFEs, WFE_scale, dt)
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

    def _eval_fused(self, num_NFEs, WFE_scale, dt):
        w = self.world.world
        st = self.state.clone()
        B = st.err.shape[0]
        reward = torch.zeros(B, dtype=torch.float32, device=st.dyn.device)
        finished = torch.zeros(B, dtype=torch.int32, device=st.dyn.device)
        j = self.judge.c_struct()
        c = self.control.c_struct() if self.control is not None else None
        w.eval_state(st.dyn, st.keys, st.err, num_NFEs, WFE_scale, dt, self.world.stages, j, c, reward, finished)
        return AbstractEnvironment(self.world, st, self.control, self.judge), reward
