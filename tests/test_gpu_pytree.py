"""World.from_bodies on the GPU: the reference's body pytrees (stand-ins with
its class and field names, tests/ref_standins.py) step bit for bit like the
build's own scenario constructors -- RoboCup with per-env ball states as a
vmapped pytree, and vmapped LunarLanders with per-env terrain, whose polygons
arrive sorted as the reference stores them (the build's constructor sorts
them on the device: the same bits)."""
import numpy as np
import pytest

import ref_standins as RS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("-m gpu test without a visible GPU (torch.cuda.is_available() is False)")
    return torch


def _same(torch, a, b):
    return torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


def test_robocup_pytree_steps_like_robocup_env(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    B = 1024
    env = pa.RoboCupEnv(batch=B, device="cuda", perturb=True)
    d = env.world.dyn.cpu().numpy()  # [nb][6][B]: the per-env ball states as vmapped leaves
    scenes = []
    for e in range(B):
        sc = RS.from_oracle(P.robocup_bodies())
        sc[4].position, sc[4].velocity = d[4, 0:2, e].copy(), d[4, 2:4, e].copy()
        sc[4].angle, sc[4].angular_velocity = d[4, 4, e].copy(), d[4, 5, e].copy()
        scenes.append(sc)
    w = pa.World.from_bodies(RS.stack(scenes), device="cuda", keys=env.world.keys.clone())
    assert w.B == B and w.geom_stride == 0 and w.scene.variant() == env.world.scene.variant()
    assert _same(torch, w.dyn, env.world.dyn) and _same(torch, w.geom, env.world.geom)
    for _ in range(3):
        w.step(16, 1e-2, pa._ffi.STAGES_ROBOCUP)
        env.world.step(16, 1e-2, pa._ffi.STAGES_ROBOCUP)
    torch.cuda.synchronize()
    assert _same(torch, w.dyn, env.world.dyn) and _same(torch, w.keys, env.world.keys)
    assert _same(torch, w.err, env.world.err)


def test_vmapped_lunar_lander_pytree_steps_like_lunar_lander(torch_cuda):
    torch = torch_cuda
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    B = 256
    tk = np.asarray(prng.split(prng.PRNGKey(0), B), np.uint32)
    ck = np.asarray(prng.split(prng.PRNGKey(1), B), np.uint32)
    i32 = lambda k: torch.tensor(k.view(np.int32), device="cuda")  # noqa: E731
    ll = pa.LunarLander(key=i32(tk), batch=B, device="cuda", collider_keys=i32(ck))
    w = pa.World.from_bodies(RS.stack([RS.from_oracle(P.lunar_lander_bodies(k)) for k in tk]), device="cuda",
                             keys=i32(ck))
    assert w.B == B and tuple(w.geom.shape) == tuple(ll.world.geom.shape)
    assert _same(torch, w.geom, ll.world.geom)  # the oracle's sort == the device sort
    assert _same(torch, w.dyn, ll.world.dyn)
    for _ in range(4):
        w.step(64, 1e-2, ll.stages)
        ll.world.step(64, 1e-2, ll.stages)
    torch.cuda.synchronize()
    assert _same(torch, w.dyn, ll.world.dyn) and _same(torch, w.keys, ll.world.keys)


def test_vmapped_per_env_body_params_vs_cport(torch_cuda):
    """A vmapped LunarLander whose lander / leg mass, inertia, elasticity and
    friction vary per env (domain randomization over the parameter leaves,
    cotix/_bodies.py:140-154; tests/penv_cases.py): World.from_bodies gives a
    per-env-parameter scene (COTIX_SCENE_PER_ENV_BODY_PARAMS) that steps bit
    for bit like the C port fed the same parameters -- state, keys, error
    bits and every contact choice -- over 3 launches of 40 fused steps."""
    torch = torch_cuda
    import parallax_amd as pa
    import penv_cases as PC
    from cotix_oracle import cport
    clib = cport.load()
    B = 512
    obs = PC.lunar_penv_bodies(B, seed=3)
    w = pa.World.from_bodies(RS.stack([RS.from_oracle(ob) for ob in obs]), device="cuda")
    assert w.scene.per_env_params and w.scene.variant()["specialization"] == "generic"
    dyn, keys = PC.state(obs)
    w.dyn.copy_(torch.tensor(dyn, device="cuda"))
    w.keys.copy_(torch.tensor(keys.view(np.int32), device="cuda"))
    sc = cport.Scene(clib, obs[0])
    G = sc.set_per_env_params(True)
    geom = PC.rows(lambda ob: cport.Scene(clib, ob).geom, obs)
    assert np.array_equal(w.geom.cpu().numpy().view(np.uint32), geom.view(np.uint32)) and G == geom.shape[1]
    want = [dyn.copy(), keys.copy(), np.zeros(B, np.uint32)]
    stages = pa._ffi.STAGES_LUNAR
    res = 0
    for _ in range(3):
        tr = {}
        w.step(40, 1e-2, stages | pa._ffi.STAGE_BROADPHASE, trace=tr)
        wch, wcl = sc.step_ex(*want, 40, stages, geom=geom, trace=True)
        torch.cuda.synchronize()
        assert np.array_equal(tr["chosen"].cpu().numpy(), wch) and np.array_equal(tr["cells"].cpu().numpy(), wcl)
        res += int((wch != np.arange(4)[None, :, None]).sum())
    got = w.dyn.cpu().numpy()
    assert np.array_equal(np.isnan(got), np.isnan(want[0]))
    assert np.array_equal(np.nan_to_num(got).view(np.uint32), np.nan_to_num(want[0]).view(np.uint32))
    assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), want[1])
    assert np.array_equal(w.err.cpu().numpy().view(np.uint32), want[2])
    assert res > B  # the parameters are exercised: resolutions in every launch
