"""env.reset() / env.step() over a batched scenario (the north-star surface;
the reference's intended env API is the non-functional
AbstractEnvironment.eval, cotix/_envs.py:37-132).

  env = BatchedEnv(RoboCupEnv(batch=4096, perturb=True))
  env.reset()
  env.step(n_steps=64)          # 64 driver steps fused in one launch
  obs = env.observation()       # f32 [B, n_bodies, 6]
"""
import torch


class BatchedEnv:
    def __init__(self, scenario, dt=1e-2, autoreset=False):
        self.scenario = scenario
        self.world = scenario.world
        self.dt = dt
        self.autoreset = autoreset
        self.resets = torch.zeros(self.world.B, dtype=torch.int32, device=self.world.device)
        self._keys0 = self.world.keys.clone()

    def reset(self):
        self.world.dyn.copy_(self.scenario.dyn_reset)
        self.world.keys.copy_(self._keys0)
        self.world.err.zero_()
        self.resets.zero_()
        return self.observation()

    def step(self, n_steps=1, action=None, action_body=None, trace=None):
        """n_steps fused driver steps; action f32 [n_steps, B, 2] is added to the
        velocity of `action_body` (default: the last body, the RoboCup ball)
        after Euler.  With autoreset an env whose error bits trip restarts from
        its reset state and keeps receiving actions.  trace: see World.step."""
        w = self.world
        body = len(w.bodies) - 1 if action_body is None else action_body
        if self.autoreset:
            w.step(n_steps, self.dt, self.scenario.stages, action=action, action_body=body,
                   dyn_reset=self.scenario.dyn_reset, resets=self.resets, trace=trace)
        else:
            w.step(n_steps, self.dt, self.scenario.stages, action=action, action_body=body, trace=trace)
        return self.observation()

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
