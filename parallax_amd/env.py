"""env.reset() / env.step() over a batched scenario (the north-star surface;
the reference's intended env API is the non-functional
AbstractEnvironment.eval, cotix/_envs.py:37-132).

  env = BatchedEnv(RoboCupEnv(batch=4096, perturb=True), autoreset=True)
  env.reset()
  obs = env.step(n_steps=64)          # 64 driver steps fused in one launch

With a device judge (parallax_amd.envs.LinearJudge) the step is an RL step:

  env = BatchedEnv(scen, judge=LinearJudge(...), autoreset=True)
  obs, reward, done = env.step(1, action=act)   # act f32 [B, 2], held over n_steps

One launch (cotix_eval) advances every env, integrates the judge's reward
rate, applies is_done / end_reward exactly as one NFE of the reference's eval
(a done env is frozen at its first done state and receives its end reward),
and writes the observation.  autoreset=True restarts an env that was done at
the previous call at the start of this one (next-step autoreset: the terminal
observation is returned once, then the env restarts from its reset state with
its key chain continuing).
"""
import numbers
from collections import namedtuple

import torch

StepResult = namedtuple("StepResult", ["obs", "reward", "done"])


class BatchedEnv:
    def __init__(self, scenario, dt=1e-2, autoreset=False, judge=None, control=None):
        self.scenario = scenario
        self.world = scenario.world
        self.dt = dt
        self.autoreset = autoreset
        w = self.world
        self.resets = torch.zeros(w.B, dtype=torch.int32, device=w.device)
        self._keys0 = w.keys.clone()
        self.judge, self.control = judge, control
        nb = len(w.bodies)
        self._obs = torch.empty(w.B, nb, 6, dtype=torch.float32, device=w.device)
        self.reward = torch.zeros(w.B, dtype=torch.float32, device=w.device)
        self.done = torch.zeros(w.B, dtype=torch.int32, device=w.device)
        self._launchers = {}

    def reset(self):
        self.world.dyn.copy_(self.scenario.dyn_reset)
        self.world.keys.copy_(self._keys0)
        self.world.err.zero_()
        self.resets.zero_()
        self.done.zero_()
        self.reward.zero_()
        return self.observation()

    def step(self, n_steps=1, *, action=None, action_body=None, trace=None, obs_out=None, copy=False):
        """n_steps fused driver steps in ONE launch; returns the observation
        f32 [B, n_bodies, 6] (written by the step kernel itself), or with a
        judge StepResult(obs, reward, done).  obs / reward / done are buffers
        of this env that the next step overwrites (no per-step allocation);
        copy=True returns clones instead (for callers that keep them, e.g. a
        trajectory list).

        action: f32 [B, 2] held over the n_steps, or [n_steps, B, 2] per step
        (no judge), added to the velocity of `action_body` (default: the last
        body, the RoboCup ball) after Euler.  Without a judge, autoreset
        restarts an env from its reset state after any step that sets its
        error bits (cotix_step_autoreset).  trace: see World.step.  obs_out: a
        caller-owned f32 [B, n_bodies, 6] tensor the kernel writes the
        observation into instead of this env's buffer (e.g. an all-gather
        send buffer)."""
        w = self.world
        if type(n_steps) is not int and (not isinstance(n_steps, numbers.Integral) or isinstance(n_steps, bool)):
            raise TypeError("n_steps must be an int (pass the action as action=...)")
        if trace is not None and self.judge is not None:
            raise ValueError("trace= is not available with a judge (the judge runs the cotix_eval program)")
        body = len(w.bodies) - 1 if action_body is None else action_body
        if self.judge is None and (trace is not None or (action is not None and action.dim() == 3)):
            if action is not None and action.dim() == 2:
                action = action[None].expand(n_steps, -1, -1)
            kw = dict(dyn_reset=self.scenario.dyn_reset, resets=self.resets) if self.autoreset else {}
            w.step(n_steps, self.dt, self.scenario.stages, action=action, action_body=body, trace=trace, **kw)
            return self.observation()  # a fresh tensor
        if action is not None and (action.dtype != torch.float32 or action.device != w.device
                                   or not action.is_contiguous()):
            action = action.to(w.device, torch.float32).contiguous()
        obs = self._obs if obs_out is None else obs_out
        launch = self._launcher(n_steps, body, obs)
        if self.judge is not None:
            self.reward.zero_()
        launch(action)
        if self.judge is None:
            return obs.clone() if copy else obs
        if copy:
            return StepResult(obs.clone(), self.reward.clone(), self.done.clone())
        return StepResult(obs, self.reward, self.done)

    def _launcher(self, n_steps, body, obs):
        """The prepared cotix_eval launch (World.eval_launcher) of a step
        configuration, built on first use: an RL loop's per-step host work is
        then one ctypes call (the launch checks only a new action's shape)."""
        w = self.world
        # everything the prepared launch copies: the public attributes by
        # value (dt, autoreset, the scenario's stages) and the judge / control
        # and the buffers by identity (a buffer swapped in by the caller, or a
        # new judge, gets its own launch).  Judges and controls are immutable
        # (envs._Frozen), and the cache entry holds them, so an id cannot be
        # reused by a later object while its launch is cached.
        key = (n_steps, body, float(self.dt), bool(self.autoreset), int(self.scenario.stages), id(self.judge),
               id(self.control), id(obs), id(w.dyn), id(w.keys), id(w.err), id(w.geom), id(self.scenario.dyn_reset))
        hit = self._launchers.get(key)
        if hit is not None:
            return hit[0]
        judge_c = self.judge.c_struct() if self.judge is not None else None
        control_c = self.control.c_struct() if self.control is not None else None
        if obs is not self._obs and (tuple(obs.shape) != tuple(self._obs.shape) or obs.dtype != torch.float32
                                     or not obs.is_contiguous() or obs.device != self._obs.device):
            raise ValueError("obs_out must be a contiguous f32 [B, n_bodies, 6] tensor on the env's device")
        if len(self._launchers) >= 8:  # (callers cycling many obs_out buffers)
            self._launchers.clear()
        if self.judge is None:
            launch = w.eval_launcher(w.dyn, w.keys, w.err, 1, n_steps, self.dt, self.scenario.stages,
                                     action_body=body, control=control_c, reset_mode=1 if self.autoreset else 0,
                                     dyn_reset=self.scenario.dyn_reset if self.autoreset else None,
                                     resets=self.resets if self.autoreset else None, obs=obs)
        else:
            launch = w.eval_launcher(w.dyn, w.keys, w.err, 1, n_steps, self.dt, self.scenario.stages,
                                     judge=judge_c, control=control_c, reward=self.reward,
                                     finished=self.done, action_body=body, reset_mode=2 if self.autoreset else 0,
                                     dyn_reset=self.scenario.dyn_reset if self.autoreset else None,
                                     resets=self.resets if self.autoreset else None, obs=obs)
        self._launchers[key] = (launch, self.judge, self.control, obs)
        return launch

    def observation(self, out=None):
        """f32 [B, n_bodies, 6] (px, py, vx, vy, angle, angular_velocity),
        contiguous, from the device transpose kernel (cotix_observe)."""
        return self.world.observe(out)

    def draw(self, painter, env=0):
        """The scenario's env.draw(painter) for env `env` (render export)."""
        return self.scenario.draw(painter, env)

    @property
    def err(self):
        return self.world.err
