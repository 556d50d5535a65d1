"""cotix_eval on the GPU (through the C-ABI): AbstractEnvironment.eval
(cotix/_envs.py:37-132) fused into one launch with the device judge /
control, and BatchedEnv.step() -> (obs, reward, done) -- against the oracle's
restatement of the reference loop (small batches, every env) and against the
kernel's host emulation at BASELINE size (4096 envs), bit for bit."""
import os
import sys

import numpy as np
import pytest

import eval_device_cases as EDC

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
F = np.float32


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a visible GPU (torch.cuda.is_available() is False)")
    return torch


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _world(torch, case):
    """A parallax_amd World of the case's scene with the case's state (GPU)."""
    import parallax_amd as pa
    from parallax_amd import bodies as PB
    from parallax_amd import shapes as PS
    ob = case["make"]()
    bodies = []
    for b in ob:
        parts = []
        for p in b.parts:
            if p.kind == "Circle":
                parts.append(PS.Circle(float(p.radius), [float(p.position[0]), float(p.position[1])]))
            else:
                parts.append(PS.AABB([float(p.lower[0]), float(p.lower[1])], [float(p.upper[0]), float(p.upper[1])]))
        bodies.append(PB.AnyBody(shape=PS.UniversalShape(*parts), mass=float(b.mass), inertia=float(b.inertia),
                                 elasticity=float(b.elasticity), friction_coefficient=float(b.friction_coefficient)))
    B = case["S0"].shape[0]
    w = pa.World(bodies, B, "cuda", torch.tensor(np.asarray(case["keys"], np.uint32).view(np.int32), device="cuda"))
    w.dyn.copy_(torch.tensor(np.ascontiguousarray(case["S0"].transpose(1, 2, 0)), device="cuda"))
    return w


@pytest.mark.parametrize("scene,name,nfe,wfe,period", [
    ("box", "x_done", 3, 10, 0.6),
    ("box", "multi", 4, 6, 0.5),
    ("robocup", "goal", 3, 4, 0.24),
    ("box", "piecewise", 4, 8, 0.64),
    ("robocup", "piecewise", 3, 5, 0.3),
])
def test_fused_eval_vs_oracle(torch_cuda, scene, name, nfe, wfe, period):
    torch = torch_cuda
    from parallax_amd import envs as E
    B = 8 if scene == "box" else 6
    case = EDC.case(scene, B, seed=5)
    w = _world(torch, case)
    j, c = EDC.device(name, case["ab"])
    state = E.WorldState(w.dyn.clone(), w.keys.clone(), w.err.clone())
    env = E.AbstractEnvironment(E.PhysicsWorld(w), state, c, j)
    assert env.fused()
    out, reward = env.eval(period, nfe, wfe)
    torch.cuda.synchronize()
    dyn = out.state.dyn.cpu().numpy()
    keys = out.state.keys.cpu().numpy().view(np.uint32)
    err = out.state.err.cpu().numpy()
    rw = reward.cpu().numpy()
    want = EDC.oracle_eval(case, name, nfe, wfe, period)
    for e, ((bodies, okey, oerr), orew, ofin) in enumerate(want):
        wd = np.array([b.dyn() for b in bodies], np.float32)
        assert same(dyn[:, :, e], wd), e
        assert np.array_equal(keys[e], okey), e
        assert int(err[e]) == int(oerr), e
        assert same(rw[e], orew), (e, rw[e], orew)
    # the product's host loop (one launch per env-step, torch judge) == the fused launch
    out2, reward2 = env.eval(period, nfe, wfe, fused=False)
    assert same(out2.state.dyn.cpu().numpy(), dyn) and same(reward2.cpu().numpy(), rw)


def test_fused_eval_4096_envs_vs_emulation(torch_cuda):
    """BASELINE size: RoboCup 4096 perturbed envs, the goal judge with the
    error trip as done, a PD control, 3 NFEs x 8 env-steps -- every env vs
    the host emulation of the same kernel program."""
    torch = torch_cuda
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    import parallax_amd as pa
    from parallax_amd import envs as E
    from cotix_oracle import physics as P
    lib = emu.load()
    scen = pa.RoboCupEnv(batch=4096, device="cuda", perturb=True)
    w = scen.world
    j, c = EDC.device("goal", 4)
    dyn0 = np.ascontiguousarray(w.dyn.cpu().numpy())
    keys0 = np.ascontiguousarray(w.keys.cpu().numpy().view(np.uint32))
    state = E.WorldState(w.dyn.clone(), w.keys.clone(), w.err.clone())
    env = E.AbstractEnvironment(E.PhysicsWorld(w), state, c, j)
    out, reward = env.eval(0.24, 3, 8)
    torch.cuda.synchronize()
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    dyn, keys, err = dyn0.copy(), keys0.copy(), np.zeros(4096, np.uint32)
    rw, fin = np.zeros(4096, np.float32), np.zeros(4096, np.uint32)
    emu.eval_(lib, h, dyn, keys, err, geom, 0, 3, 8, float(F(F(0.24 / 3) / F(8.0))), 1 | 4 | 16, judge=j.c_struct(),
              control=c.c_struct(), reward=rw, finished=fin)
    assert same(out.state.dyn.cpu().numpy(), dyn)
    assert np.array_equal(out.state.keys.cpu().numpy().view(np.uint32), keys)
    assert same(reward.cpu().numpy(), rw)
    assert fin.sum() > 100  # RoboCup's error trip ends most episodes (done_on_error)


def test_batched_env_rl_loop_vs_emulation(torch_cuda):
    """BatchedEnv(judge, autoreset).step(action) -> (obs, reward, done), 20
    calls of 2 env-steps on 4096 RoboCup envs: obs, reward, done, state,
    keys and restart counts equal the emulated kernel's, every call."""
    torch = torch_cuda
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    import parallax_amd as pa
    from cotix_oracle import physics as P
    lib = emu.load()
    B = 4096
    j, _ = EDC.device("goal", 4)
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True), judge=j, autoreset=True)
    env.reset()
    w = env.world
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    dyn = np.ascontiguousarray(w.dyn.cpu().numpy())
    reset = dyn.copy()
    keys = np.ascontiguousarray(w.keys.cpu().numpy().view(np.uint32))
    err, fin, resets = np.zeros(B, np.uint32), np.zeros(B, np.uint32), np.zeros(B, np.uint32)
    gen = torch.Generator().manual_seed(0)
    total_done = 0
    for q in range(20):
        act = (torch.randn(B, 2, generator=gen) * 0.5).to("cuda")
        obs, reward, done = env.step(2, action=act)
        rw = np.zeros(B, np.float32)
        emu.eval_(lib, h, dyn, keys, err, geom, 0, 1, 2, 1e-2, 1 | 4 | 16, judge=j.c_struct(),
                  action=np.ascontiguousarray(act.cpu().numpy()), action_body=4, reward=rw, finished=fin,
                  reset_mode=2, dyn_reset=reset, resets=resets)
        torch.cuda.synchronize()
        assert same(obs.cpu().numpy(), dyn.transpose(2, 0, 1)), q
        assert same(reward.cpu().numpy(), rw), q
        assert np.array_equal(done.cpu().numpy().astype(np.uint32), fin), q
        total_done += int(fin.sum())
    assert same(w.dyn.cpu().numpy(), dyn)
    assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(env.resets.cpu().numpy().astype(np.uint32), resets)
    assert total_done > 0 and resets.sum() > 0


def test_step_obs_from_kernel_equals_observe(torch_cuda):
    """BatchedEnv.step() without a judge: one launch (restart on error,
    observation written by the step kernel) == cotix_step_autoreset +
    cotix_observe on a twin env."""
    torch = torch_cuda
    import parallax_amd as pa
    a = pa.BatchedEnv(pa.RoboCupEnv(batch=1000, device="cuda", perturb=True), autoreset=True)
    b = pa.BatchedEnv(pa.RoboCupEnv(batch=1000, device="cuda", perturb=True), autoreset=True)
    a.reset()
    b.reset()
    outs = [torch.full((1000, 5, 6), 7.0, device="cuda") for _ in range(2)]
    for i in range(7):
        # odd steps: into a caller's buffer (the bench's all-gather send buffers)
        o = a.step(3, obs_out=outs[i % 2]) if i % 2 else a.step(3)
        if i % 2:
            assert o.data_ptr() == outs[1].data_ptr()
        b.world.step(3, 1e-2, b.scenario.stages, dyn_reset=b.scenario.dyn_reset, resets=b.resets)
        ob = b.observation()
        torch.cuda.synchronize()
        assert torch.equal(o.view(torch.int32), ob.view(torch.int32))
    assert torch.equal(a.resets, b.resets) and int(a.resets.sum()) > 0
    assert bool((outs[0] == 7.0).all())  # never written
    with pytest.raises(ValueError):
        a.step(1, obs_out=torch.empty(999, 5, 6, device="cuda"))


def test_step_launch_follows_env_attributes(torch_cuda):
    """BatchedEnv.step's prepared launch is rebuilt when a public attribute it
    copies changes between steps (dt, autoreset, the scenario's stages): each
    step equals the same step of a twin env driven through World.step with
    the attribute's current value."""
    torch = torch_cuda
    import parallax_amd as pa
    from parallax_amd import _ffi
    a = pa.BatchedEnv(pa.RoboCupEnv(batch=512, device="cuda", perturb=True), autoreset=True)
    b = pa.BatchedEnv(pa.RoboCupEnv(batch=512, device="cuda", perturb=True), autoreset=True)
    a.reset()
    b.reset()
    plan = [(1e-2, True, None), (5e-3, True, None), (5e-3, False, None), (2e-2, True, _ffi.STAGE_EULER),
            (1e-2, True, None)]
    stages0 = a.scenario.stages
    for dt, ar, st in plan:
        a.dt, a.autoreset = dt, ar
        a.scenario.stages = stages0 if st is None else st
        o = a.step(2)
        kw = dict(dyn_reset=b.scenario.dyn_reset, resets=b.resets) if ar else {}
        b.world.step(2, dt, stages0 if st is None else st, **kw)
        ob = b.observation()
        torch.cuda.synchronize()
        assert torch.equal(o.view(torch.int32), ob.view(torch.int32)), (dt, ar, st)
    a.scenario.stages = stages0
