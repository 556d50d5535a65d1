"""The kernel's host emulation under AddressSanitizer + UBSan (standalone
executable tests/emu/build/asan_driver; GPU sanitizers are unavailable on
this pool): the fused step (every envs-per-wave variant, incl. the
wave-cooperative phase C) and the differentiable rollout + backward, on the
RoboCup, LunarLander and box-world scenes.  The sanitized run must exit
cleanly and agree bit for bit with the plain emulation."""
import os
import subprocess

import numpy as np
import pytest

import grad_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "emu", "build", "asan_driver")
TYPE_ID = {"Circle": 0, "AABB": 1, "Polygon": 2, "Polygon3": 3, "Polygon4": 4, "Polygon5": 5, "Polygon6": 6}


@pytest.fixture(scope="module")
def emu_mod():
    import sys
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so", "build/asan_driver"],
                   check=True)
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    return emu, emu.load()


def _scene_arrays(bodies):
    params = np.array([[b.mass, b.inertia, b.elasticity, b.friction_coefficient] for b in bodies], np.float32)
    pb, pt, pn, geom = [], [], [], []
    for i, b in enumerate(bodies):
        for p in b.parts:
            pb.append(i)
            pt.append(TYPE_ID[p.kind])
            if p.kind == "Circle":
                pn.append(0)
                geom += [p.radius, p.position[0], p.position[1], 0.0]
            elif p.kind == "AABB":
                pn.append(0)
                geom += [p.lower[0], p.lower[1], p.upper[0], p.upper[1]]
            else:
                pn.append(len(p.vertices_))
                for v in p.vertices_:
                    geom += [v[0], v[1]]
    return params, np.array(pb, np.int32), np.array(pt, np.int32), np.array(pn, np.int32), np.array(geom, np.float32)


def _run_driver(tmp_path, bodies, dyn, keys, T, stages, E, mode=0, actions=None, ab=0, w=None):
    params, pb, pt, pn, geom = _scene_arrays(bodies)
    nb, B = dyn.shape[0], dyn.shape[2]
    inp, out = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    with open(inp, "wb") as f:
        np.array([nb, len(pb), B, T, stages, len(geom), 0, mode, E, ab], np.int32).tofile(f)
        for x in (params, pb, pt, pn, geom, dyn.astype(np.float32), keys.astype(np.uint32)):
            np.ascontiguousarray(x).tofile(f)
        if mode == 1:
            np.ascontiguousarray(actions, np.float32).tofile(f)
            np.ascontiguousarray(w, np.float32).tofile(f)
    r = subprocess.run([DRIVER, inp, out], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    raw = np.fromfile(out, np.uint8)
    return raw, geom


@pytest.mark.parametrize("E", [1, 2, 4, 8])
def test_asan_robocup_step(emu_mod, tmp_path, E):
    emu, lib = emu_mod
    from cotix_oracle import cport
    B, T = 24, 12
    dyn, keys = cport.robocup_batch(B)
    raw, _ = _run_driver(tmp_path, GC.P.robocup_bodies(), dyn, keys, T, 1 | 4 | 16, E)
    h, geom = emu.oracle_scene(lib, GC.P.robocup_bodies())
    d, k, err = dyn.copy(), keys.copy(), np.zeros(B, np.uint32)
    emu.step(lib, h, d, k, err, geom, 0, T, 1 | 4 | 16, E=E)
    want = np.concatenate([d.reshape(-1).view(np.uint8), k.reshape(-1).view(np.uint8), err.view(np.uint8)])
    assert np.array_equal(raw, want)


def test_asan_lunar_step(emu_mod, tmp_path):
    emu, lib = emu_mod
    from cotix_oracle import prng
    bodies = GC.P.lunar_lander_bodies(prng.PRNGKey(0))
    B, T = 8, 6
    base = np.array([b.dyn() for b in bodies], np.float32)
    dyn = np.ascontiguousarray(np.repeat(base[:, :, None], B, axis=2))
    dyn[0, 1, ::2] -= 6.2  # half the landers start in contact with the terrain
    keys = np.asarray(prng.split(prng.PRNGKey(1), B), np.uint32)
    raw, _ = _run_driver(tmp_path, bodies, dyn, keys, T, 31, 4)
    h, geom = emu.oracle_scene(lib, bodies)
    d, k, err = dyn.copy(), keys.copy(), np.zeros(B, np.uint32)
    emu.step(lib, h, d, k, err, geom, 0, T, 31, E=4)
    want = np.concatenate([d.reshape(-1).view(np.uint8), k.reshape(-1).view(np.uint8), err.view(np.uint8)])
    assert np.array_equal(raw, want)


@pytest.mark.parametrize("E", [1, 4])
def test_asan_box_world_rollout_backward(emu_mod, tmp_path, E):
    emu, lib = emu_mod
    B, T = 8, 16
    case = GC.box_case(B, T, seed=2)
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    raw, _ = _run_driver(tmp_path, case["make"](), dyn, case["keys"], T, 21, E, mode=1, actions=case["actions"],
                         ab=case["ab"], w=case["w"])
    h, geom = emu.oracle_scene(lib, case["make"]())
    d, k, err = dyn.copy(), np.array(case["keys"], np.uint32, copy=True), np.zeros(B, np.uint32)
    ret, sd, sk, tape = emu.rollout(lib, h, d, k, err, geom, 0, 21, case["actions"], case["ab"], case["w"], E=E)
    ga, gd = emu.rollout_backward(lib, h, sd, sk, geom, 0, 21, case["actions"], case["ab"], case["w"], E=E,
                                  tape=tape)
    want = np.concatenate([x.reshape(-1).view(np.uint8) for x in (d, k, err, ret, ga, gd)])
    assert np.array_equal(raw, want)


@pytest.mark.parametrize("scene", ["lunar", "poly_box"])
def test_asan_polygon_rollout_backward(emu_mod, tmp_path, scene):
    """The polygon gradients (phase GE's GJK/EPA contact VJPs, the joints in
    phase G) under the sanitizers."""
    emu, lib = emu_mod
    if scene == "lunar":
        case, stages = GC.lunar_case(4, 8, seed=1), 1 | 2 | 4 | 8 | 16 | 32
    else:
        case, stages = GC.poly_box_case(4, 8, seed=1), 1 | 4 | 16
    B, T = case["S0"].shape[0], case["actions"].shape[0]
    dyn = np.ascontiguousarray(case["S0"].transpose(1, 2, 0))
    raw, _ = _run_driver(tmp_path, case["make"](), dyn, case["keys"], T, stages, 4, mode=1,
                         actions=case["actions"], ab=case["ab"], w=case["w"])
    h, geom = emu.oracle_scene(lib, case["make"]())
    d, k, err = dyn.copy(), np.array(case["keys"], np.uint32, copy=True), np.zeros(B, np.uint32)
    ret, sd, sk, tape = emu.rollout(lib, h, d, k, err, geom, 0, stages, case["actions"], case["ab"], case["w"], E=4)
    ga, gd = emu.rollout_backward(lib, h, sd, sk, geom, 0, stages, case["actions"], case["ab"], case["w"], E=4,
                                  tape=tape)
    want = np.concatenate([x.reshape(-1).view(np.uint8) for x in (d, k, err, ret, ga, gd)])
    assert np.array_equal(raw, want)
