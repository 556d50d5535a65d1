"""The reference's own body pytrees into a World (parallax_amd.pytree,
World.from_bodies), on CPU: stand-in objects with the reference's class and
field names (tests/ref_standins.py), filled from the oracle's restatement of
the reference constructors, give the same scene, geometry and state as the
build's own scenario constructors -- bit for bit -- single and vmapped."""
import numpy as np
import pytest
import torch

import ref_standins as RS


def _same(a, b):
    return torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


def test_robocup_bodies_drop_in():
    import parallax_amd as pa
    from cotix_oracle import physics as P
    w = pa.World.from_bodies(RS.from_oracle(P.robocup_bodies()), batch=8, device="cpu")
    ref = pa.World(pa.scenarios.robocup_bodies(), 8, "cpu")
    assert w.B == 8
    assert w.scene.variant() == ref.scene.variant() == {"envs_per_wave": 4, "specialization": "robocup"}
    assert [b.params() for b in w.bodies] == [b.params() for b in ref.bodies]
    assert [b.is_area for b in w.bodies] == [b.is_area for b in ref.bodies]
    assert _same(w.dyn, ref.dyn) and _same(w.geom, ref.geom)


def test_robocup_env_object_and_vmapped_ball_state():
    """An env object (its .bodies), and a vmapped pytree whose ball state
    differs per env: the env axis comes from the leaves."""
    import parallax_amd as pa
    from cotix_oracle import physics as P

    class Env:  # RoboCupEnv().bodies (cotix/_robocup.py:124-130)
        bodies = RS.from_oracle(P.robocup_bodies())
    assert _same(pa.World.from_bodies(Env(), device="cpu").dyn, pa.World(pa.scenarios.robocup_bodies(), 1, "cpu").dyn)
    rng = np.random.default_rng(0)
    scenes = []
    for e in range(5):
        sc = RS.from_oracle(P.robocup_bodies())
        sc[4].position = rng.uniform(-4, 4, 2).astype(np.float32)
        sc[4].angular_velocity = np.float32(rng.uniform(-10, 10))
        scenes.append(sc)
    w = pa.World.from_bodies(RS.stack(scenes), device="cpu")
    assert w.B == 5 and w.geom.dim() == 1  # shared geometry stays shared
    for e in range(5):
        assert torch.equal(w.dyn[4, 0:2, e], torch.tensor(scenes[e][4].position))
        assert float(w.dyn[4, 5, e]) == float(scenes[e][4].angular_velocity)


def test_lunar_lander_bodies_drop_in(emu_geom):
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    ob = P.lunar_lander_bodies(prng.PRNGKey(0))
    w = pa.World.from_bodies(RS.from_oracle(ob), device="cpu")
    assert w.scene.variant() == {"envs_per_wave": 4, "specialization": "lunar"}
    assert np.array_equal(w.geom.numpy().view(np.uint32), emu_geom(ob).view(np.uint32))
    assert np.array_equal(w.dyn[:, :, 0].numpy(), np.array([b.dyn() for b in ob], np.float32))
    assert [b.params() for b in w.bodies] == [[float(b.mass), float(b.inertia), float(b.elasticity),
                                              float(b.friction_coefficient)] for b in ob]


def test_vmapped_lunar_landers(emu_geom):
    """jax.vmap(lambda k: LunarLander(k).bodies)(keys): per-env terrain as a
    leading batch dimension of the terrain quads' vertices."""
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    keys = [np.asarray(k, np.uint32) for k in prng.split(prng.PRNGKey(7), 6)]
    obs = [P.lunar_lander_bodies(k) for k in keys]
    w = pa.World.from_bodies(RS.stack([RS.from_oracle(ob) for ob in obs]), device="cpu")
    assert w.B == 6 and tuple(w.geom.shape) == (6, w.scene.geom_floats)
    for e, ob in enumerate(obs):
        assert np.array_equal(w.geom[e].numpy().view(np.uint32), emu_geom(ob).view(np.uint32)), e


def test_adapter_errors():
    import parallax_amd as pa
    from cotix_oracle import physics as P
    sc = RS.from_oracle(P.robocup_bodies())

    class Ellipse:
        pass
    bad = RS.from_oracle(P.robocup_bodies())
    bad[4].shape.parts = [Ellipse()]
    with pytest.raises(TypeError, match="Ellipse is not in the contact-function registry"):
        pa.World.from_bodies(bad, device="cpu")
    two = RS.stack([RS.from_oracle(P.robocup_bodies()) for _ in range(2)])
    two[4].mass = np.array([0.5, 0.6], np.float32)  # a varying parameter leaf: per-env parameters
    w2 = pa.World.from_bodies(two, device="cpu")
    assert w2.scene.per_env_params and tuple(w2.geom.shape) == (2, w2.scene.geom_floats)
    two[4].mass = np.array([[0.5], [0.6]], np.float32)
    with pytest.raises(ValueError, match="expected rank 0"):
        pa.World.from_bodies(two, device="cpu")
    with pytest.raises(ValueError, match="batch"):
        pa.World.from_bodies(RS.stack([sc, RS.from_oracle(P.robocup_bodies())]), batch=3, device="cpu")

    class NotABody:
        shape = None
    with pytest.raises(TypeError, match="lacks the AnyBody fields"):
        pa.World.from_bodies([NotABody()], device="cpu")


@pytest.fixture(scope="module")
def emu_geom():
    """The local geometry words of oracle bodies as the scene compiler lays
    them out (the host emulation's oracle_scene: test infrastructure)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu"))
    import emu
    lib = emu.load()
    return lambda bodies: emu.oracle_scene(lib, bodies)[1]
