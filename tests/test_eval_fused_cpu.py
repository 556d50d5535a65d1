"""cotix_eval -- AbstractEnvironment.eval (cotix/_envs.py:37-132) fused into
one launch with a device judge / control -- on CPU through the kernel's host
emulation: against the oracle's restatement of the reference loop
(oracle/cotix_oracle/envs.py) bit for bit (state, key, err, reward,
finished), against the product's own host loop over the same judge (torch
methods), the env.step() RL loop with next-step autoreset, and the
observation / restart-on-error path the bench's K = 1 line uses."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import eval_device_cases as EDC
import grad_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))
F = np.float32


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    return emu, emu.load()


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _state(case):
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0)).astype(np.float32)
    keys = np.array(case["keys"], np.uint32)  # a copy: the kernel advances keys in place
    return dyn, keys, np.zeros(dyn.shape[2], np.uint32)


def _check_vs_oracle(dyn, keys, err, reward, fin, want):
    for e, ((bodies, okey, oerr), orew, ofin) in enumerate(want):
        w = np.array([b.dyn() for b in bodies], np.float32)
        assert same(dyn[:, :, e], w), (e, dyn[:, :, e], w)
        assert np.array_equal(keys[e], okey), e
        assert int(err[e]) == int(oerr), (e, err[e], oerr)
        assert same(reward[e], orew), (e, reward[e], orew)
        assert bool(fin[e]) == bool(ofin), (e, fin[e], ofin)


@pytest.mark.parametrize("scene,name,nfe,wfe,period", [
    ("box", "x_done", 3, 10, 0.6),
    ("box", "multi", 4, 6, 0.5),
    ("robocup", "goal", 3, 4, 0.24),
    ("box", "piecewise", 4, 8, 0.64),
    ("robocup", "piecewise", 3, 5, 0.3),
    ("robocup", "x_done", 2, 5, 0.2),
])
@pytest.mark.parametrize("EW", [1, 4])
def test_fused_eval_vs_oracle(emu_lib, scene, name, nfe, wfe, period, EW):
    emu, lib = emu_lib
    B = 8 if scene == "box" else 6
    case = EDC.case(scene, B, seed=5)
    ab = case["ab"]
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn, keys, err = _state(case)
    reward, fin = np.zeros(B, np.float32), np.zeros(B, np.uint32)
    j, c = EDC.device(name, ab)
    tpn = F(period / nfe)
    dt = float(F(tpn / F(float(wfe))))
    emu.eval_(lib, h, dyn, keys, err, geom, 0, nfe, wfe, dt, 1 | 4 | 16, judge=j.c_struct(), control=c.c_struct(),
              reward=reward, finished=fin, E=EW)
    want = EDC.oracle_eval(case, name, nfe, wfe, period)
    _check_vs_oracle(dyn, keys, err, reward, fin, want)
    if scene == "box":
        assert fin.sum() >= 2  # envs frozen mid-eval and at the start are covered
    if name == "goal":
        assert fin.sum() >= 1  # the error trip ends episodes (done_on_error)


@pytest.mark.parametrize("name", ["multi", "piecewise"])
def test_fused_eval_equals_product_host_loop(emu_lib, name):
    """The product's generic eval loop (one launch per env-step, judge and
    control evaluated by their torch methods) == the fused launch, bit for
    bit: the LinearJudge / AffineControl torch methods are the kernel's
    expressions (piecewise: the rate's pieces per region, the clipped
    control)."""
    emu, lib = emu_lib
    from parallax_amd import envs as E
    from test_envs_cpu import EmuWorld
    B = 8
    case = EDC.case("box", B, seed=5)
    ab = case["ab"]
    j, c = EDC.device(name, ab)
    world = EmuWorld(emu, lib, case["make"](), 1 | 4 | 16)
    dyn, keys, err = _state(case)
    state = E.WorldState(torch.from_numpy(dyn.copy()), torch.from_numpy(keys.view(np.int32).copy()),
                         torch.zeros(B, dtype=torch.int32))
    env = E.AbstractEnvironment(world, state, c, j)
    assert not env.fused()  # EmuWorld is not a PhysicsWorld: the host loop runs
    out, reward = env.eval(0.5, 4, 6)
    h, geom = world.h, world.geom
    rw, fin = np.zeros(B, np.float32), np.zeros(B, np.uint32)
    emu.eval_(lib, h, dyn, keys, err, geom, 0, 4, 6, float(F(F(0.5 / 4) / F(6.0))), 1 | 4 | 16,
              judge=j.c_struct(), control=c.c_struct(), reward=rw, finished=fin)
    assert same(out.state.dyn.numpy(), dyn)
    assert np.array_equal(out.state.keys.numpy().view(np.uint32), keys)
    assert same(reward.numpy(), rw)


def test_env_step_rl_loop_next_step_autoreset(emu_lib):
    """BatchedEnv.step(action) semantics: each call is one NFE of wfe
    env-steps with the action held; a done env is frozen at its first done
    state with its end reward, and restarts from its reset state at the next
    call (next-step autoreset, key chain continuing) -- vs the oracle loop."""
    emu, lib = emu_lib
    from cotix_oracle import envs as OE
    B, wfe, calls = 8, 3, 6
    case = EDC.case("box", B, seed=7)
    ab = case["ab"]
    jn = EDC.judges("multi", ab)[0]
    from parallax_amd import envs as E
    j = E.LinearJudge(**jn)
    oj = OE.LinearJudge(**jn)
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn, keys, err = _state(case)
    reset = dyn.copy()
    fin, resets = np.zeros(B, np.uint32), np.zeros(B, np.uint32)
    rng = np.random.default_rng(3)
    acts = (rng.normal(size=(calls, B, 2)) * 0.3).astype(np.float32)
    # oracle side
    ost = []
    for e in range(B):
        bodies = case["make"]()
        for b, row in zip(bodies, case["S0"][e]):
            b.set_dyn(row)
        ost.append([(bodies, np.asarray(case["keys"][e], np.uint32), 0), False, 0])
    for q in range(calls):
        rw = np.zeros(B, np.float32)
        emu.eval_(lib, h, dyn, keys, err, geom, 0, 1, wfe, 1e-2, 1 | 4 | 16, judge=j.c_struct(),
                  action=np.ascontiguousarray(acts[q]), action_body=ab, reward=rw, finished=fin, reset_mode=2,
                  dyn_reset=reset, resets=resets)
        for e in range(B):
            st, ofin, ores = ost[e]
            if ofin:  # next-step autoreset: reset state, key chain continues, err cleared
                bodies = case["make"]()
                for b, row in zip(bodies, case["S0"][e]):
                    b.set_dyn(row)
                st, ofin, ores = (bodies, st[1], 0), False, ores + 1
            st, orew, ofin = OE.eval_env(case["step"], st, OE.HeldImpulse(acts[q, e]), oj, F(wfe * 1e-2) * 1.0, 1,
                                         wfe, GC.D0, ab, carry=(0.0, False))
            ost[e] = [st, ofin, ores]
            w = np.array([b.dyn() for b in st[0]], np.float32)
            assert same(dyn[:, :, e], w), (q, e)
            assert np.array_equal(keys[e], st[1]), (q, e)
            assert same(rw[e], orew), (q, e, rw[e], orew)
            assert bool(fin[e]) == ofin and int(resets[e]) == ores, (q, e)
    assert resets.sum() >= 1 and fin.sum() + resets.sum() >= 2


def test_eval_obs_and_restart_on_error_equals_step(emu_lib):
    """judge = NULL, reset_mode 1, obs: the launch BatchedEnv.step() / the
    bench's K = 1 line use == cotix_step_autoreset + the transpose."""
    emu, lib = emu_lib
    case = EDC.case("robocup", 16, seed=1)
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn, keys, err = _state(case)
    reset = dyn.copy()
    d2, k2, e2 = dyn.copy(), keys.copy(), err.copy()
    r1, r2 = np.zeros(16, np.uint32), np.zeros(16, np.uint32)
    obs = np.full((16, 5, 6), np.nan, np.float32)
    for _ in range(5):
        emu.eval_(lib, h, dyn, keys, err, geom, 0, 1, 3, 1e-2, 1 | 4 | 16, reset_mode=1, dyn_reset=reset, resets=r1,
                  obs=obs)
        emu.step(lib, h, d2, k2, e2, geom, 0, 3, 1 | 4 | 16, E=4, dyn_reset=reset, resets=r2)
        assert same(obs, dyn.transpose(2, 0, 1))
    assert same(dyn, d2) and np.array_equal(keys, k2) and np.array_equal(err, e2) and np.array_equal(r1, r2)
    assert r1.sum() > 0


def test_eval_argument_errors(emu_lib):
    emu, lib = emu_lib
    case = EDC.case("box", 4)
    h, geom = emu.oracle_scene(lib, case["make"]())
    dyn, keys, err = _state(case)
    from parallax_amd import envs as E
    j = E.LinearJudge(rate_w={0: 1.0})
    with pytest.raises(RuntimeError):  # a judge needs reward + finished
        emu.eval_(lib, h, dyn, keys, err, geom, 0, 1, 1, 1e-2, 21, judge=j.c_struct())
    bad = E.LinearJudge(rate_w={7 * 6 + 1: 1.0})  # weight beyond the scene's 7 bodies
    with pytest.raises(RuntimeError):
        emu.eval_(lib, h, dyn, keys, err, geom, 0, 1, 1, 1e-2, 21, judge=bad.c_struct(),
                  reward=np.zeros(4, np.float32), finished=np.zeros(4, np.uint32))
    with pytest.raises(ValueError):
        E.LinearJudge(rate_w={k: 1.0 for k in range(17)})


def test_judge_and_control_are_immutable():
    """a prepared launch copies the device struct once, so an
    in-place change must raise instead of reaching a stale launch."""
    import pytest
    from parallax_amd.envs import AffineControl, LinearJudge
    j = LinearJudge(rate_w={2: 0.1}, rate_regions=[(0, [-1.0] * 6, [1.0] * 6, {0: 1.0}, 0.5)])
    c = AffineControl(0, gain=[[1.0] * 6, [0.0] * 6], clip=((-1, 1), (-2, 2)))
    for obj, attr in ((j, "rate_regions"), (j, "done_on_error"), (c, "clip"), (c, "gain")):
        with pytest.raises(AttributeError):
            setattr(obj, attr, getattr(obj, attr))
    with pytest.raises(TypeError):
        c.gain[0][0] = 2.0  # nested rows are tuples
    assert c.c_struct().saturate == 1 and j.c_struct().n_rate_regions == 1
