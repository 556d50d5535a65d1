"""CPU-side checks of the drop-in boundary: the HIP library loads, exports
every symbol include/cotix_amd.h declares, the scene compiler reproduces the
collider's trace-time enumeration (cotix/_colliders.py:86-131), and the
scenario constants equal the oracle's.  No kernel is launched."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "cotix_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(cotix_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    import parallax_amd as pa
    syms = declared_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(pa._ffi.lib, s), s
        assert s in pa._ffi.SIGNATURES, s
    assert pa._ffi.lib.cotix_version().startswith(b"cotix_amd")


def test_robocup_scene_tables():
    import parallax_amd as pa
    s = pa.Scene(pa.scenarios.robocup_bodies())
    # 22x22 AABB candidates with i >= j (475) + 8x8 Circle/AABB (64); 9 + 9 + 13 +
    # 9 distinct part pairs; cells (1,0),(1,1),(2,0),(2,1),(2,2),(3,0),(3,1),(3,2),(4,0..3)
    assert s.info() == {"contacts": 40, "cells": 12, "candidates": 539, "types": 2}
    assert s.geom_floats == 8 * 4 + 4


def test_lunar_scene_tables():
    import parallax_amd as pa
    s = pa.Scene(pa.scenarios.lunar_lander_bodies(torch.zeros(1, 7, 4, 2)))
    # (P4,P6): 9x9 -> 81, (P4,P4): 15x15 -> 225; 306 candidates, all with i >= j
    assert s.info() == {"contacts": 25, "cells": 7, "candidates": 306, "types": 2}
    assert s.geom_floats == 12 + 8 + 8 + 7 * 8


def test_illegal_pair_is_rejected():
    import parallax_amd as pa
    bodies = [pa.AnyBody(shape=pa.UniversalShape(pa.AABB([0, 0], [1, 1]))),
              pa.AnyBody(shape=pa.UniversalShape(pa.Polygon3([[0, 0], [1, 0], [0, 1]])))]
    with pytest.raises(RuntimeError, match="illegal shape pair"):
        pa.Scene(bodies)


def test_robocup_constants_match_oracle():
    import parallax_amd as pa
    from cotix_oracle import physics as P
    ours = pa.scenarios.robocup_bodies()
    ref = P.robocup_bodies()
    for a, b in zip(ours, ref):
        assert a.params() == [float(b.mass), float(b.inertia), float(b.elasticity), float(b.friction_coefficient)]
        assert np.array_equal(a.dyn_columns(1)[:, 0].numpy(), np.array(b.dyn(), np.float32))
        for pa_, pb_ in zip(a.shape.parts, b.parts):
            g = pa_.local_geometry().numpy()
            if pb_.kind == "AABB":
                want = np.array([*pb_.lower, *pb_.upper], np.float32)
            else:
                want = np.array([pb_.radius, *pb_.position, 0.0], np.float32)
            assert np.array_equal(g, want)


def test_lunar_leg_constants_match_oracle():
    import parallax_amd as pa
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    ref = P.lunar_lander_bodies(prng.PRNGKey(0))
    assert np.array_equal(pa.scenarios.RIGHT_LEG, np.array(ref[1].parts[0].vertices_, np.float32))
    assert np.array_equal(pa.scenarios.LEFT_LEG, np.array(ref[2].parts[0].vertices_, np.float32))
    ours = pa.scenarios.lunar_lander_bodies(torch.zeros(1, 7, 4, 2))
    for a, b in zip(ours[:3], ref[:3]):
        assert a.params() == [float(b.mass), float(b.inertia), float(b.elasticity), float(b.friction_coefficient)]
        assert np.array_equal(a.dyn_columns(1)[:, 0].numpy(), np.array(b.dyn(), np.float32))


def test_product_path_does_not_import_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "parallax_amd")):
        for f in files:
            if f.endswith(".py"):
                assert "cotix_oracle" not in open(os.path.join(dirpath, f)).read(), f


def _robocup_world_cpu(B=4):
    """A RoboCup World whose tensors live on the CPU: the host-side argument
    checks below fail before anything is launched."""
    import parallax_amd as pa
    return pa.World(pa.scenarios.robocup_bodies(), B, "cpu", torch.zeros(B, 2, dtype=torch.int32))


def test_release_library_has_no_debug_or_variant_env_knobs():
    """The release library reads no environment variable that changes what a
    launch computes or which kernel runs: phase skips exist only in the
    tooling build (-DCOTIX_TOOLING), kernel variants are cotix_scene_set_variant."""
    import parallax_amd as pa
    blob = open(pa._ffi.LIB_PATH, "rb").read()
    for name in (b"COTIX_DEBUG_SKIP", b"COTIX_ENVS_PER_WAVE", b"COTIX_NO_SPEC"):
        assert name not in blob, name


def test_scene_variant_api():
    import parallax_amd as pa
    s = pa.Scene(pa.scenarios.robocup_bodies())
    assert s.variant() == {"envs_per_wave": 4, "specialization": "robocup"}
    s.set_variant(4, False)
    assert s.variant() == {"envs_per_wave": 4, "specialization": "generic"}
    s.set_variant(2)
    assert s.variant() == {"envs_per_wave": 2, "specialization": "robocup"}  # specializations: 4 and 2 envs per wave
    s.set_variant(8)
    assert s.variant() == {"envs_per_wave": 8, "specialization": "generic"}
    s.set_variant(0)
    assert s.variant()["envs_per_wave"] == 4
    with pytest.raises(RuntimeError, match="envs_per_wave"):
        s.set_variant(3)
    # the specializations fold the whole header: the default constants per PRNG layout
    s = pa.Scene(pa.scenarios.robocup_bodies(), params=pa.Params(prng_layout="partitionable"))
    assert s.variant()["specialization"] == "robocup_partitionable"
    s = pa.Scene(pa.scenarios.robocup_bodies(), params=pa.Params(contact_p=0.25))
    assert s.variant()["specialization"] == "generic"
    # the box world's structure is specialized at 4 envs per wave only (the
    # launcher's table): at 2 the generic kernel runs and is reported
    s = pa.Scene(pa.scenarios.box_world_bodies())
    assert s.variant()["specialization"] == "box"
    s.set_variant(2)
    assert s.variant() == {"envs_per_wave": 2, "specialization": "generic"}
    s.set_variant(1)
    assert s.variant()["specialization"] == "generic"


def test_eval_rejects_reset_mode2_without_judge_and_overflow():
    """cotix_eval: reset_mode 2 restarts the envs the judge finished, so it
    needs a judge (else `finished` is never cleared); n_nfe * wfe must not
    overflow int.  Both fail in the argument checks, before any launch."""
    import ctypes
    import parallax_amd as pa
    lib = pa._ffi.lib
    s = pa.Scene(pa.scenarios.robocup_bodies())
    fake = ctypes.c_void_p(4096)  # never dereferenced: the checks fail first
    rc = lib.cotix_eval(s.handle, fake, fake, fake, fake, 0, 8, 1, 4, 1e-2, pa._ffi.STAGES_ROBOCUP, None, None,
                        None, 0, None, fake, 2, fake, None, None, None)
    assert rc != 0 and b"needs a judge" in lib.cotix_last_error()
    rc = lib.cotix_eval(s.handle, fake, fake, fake, fake, 0, 8, 1 << 16, 1 << 16, 1e-2, pa._ffi.STAGES_ROBOCUP,
                        None, None, None, 0, None, None, 0, None, None, None, None)
    assert rc != 0 and b"overflows" in lib.cotix_last_error()


def test_eval_state_checks_dtypes():
    w = _robocup_world_cpu()
    bad = torch.zeros(w.B, dtype=torch.float64)
    with pytest.raises(ValueError, match="dtype"):
        w.eval_state(w.dyn, w.keys, w.err, 1, 1, 1e-2, 21, reward=bad)
    with pytest.raises(ValueError, match="dtype"):
        w.eval_state(w.dyn, w.keys, w.err, 1, 1, 1e-2, 21, finished=torch.zeros(w.B, dtype=torch.int64))
    with pytest.raises(ValueError, match="dtype"):
        w.eval_state(w.dyn, w.keys.to(torch.int64), w.err, 1, 1, 1e-2, 21)


def test_env_step_argument_checks():
    import parallax_amd as pa
    from parallax_amd import envs as E

    class Scen:
        world = _robocup_world_cpu()
        dyn_reset = world.dyn.clone()
        stages = pa._ffi.STAGES_ROBOCUP

    env = pa.BatchedEnv(Scen())
    with pytest.raises(TypeError, match="n_steps"):
        env.step(torch.zeros(4, 2))  # the action passed positionally
    envj = pa.BatchedEnv(Scen(), judge=E.LinearJudge(rate_w={24: 1.0}))
    with pytest.raises(ValueError, match="trace"):
        envj.step(1, trace={})


def test_prepared_eval_launch_marshals_every_argument(monkeypatch):
    """World.eval_launcher / BatchedEnv.step's prepared launch: every argument
    converts through cotix_eval's declared ctypes signature (checked with the
    real argtypes; the call itself is stubbed -- no GPU here), the action slot
    is swapped per launch, and the launch is reused for the same buffers."""
    import ctypes
    import parallax_amd as pa
    from parallax_amd import envs as E
    real = pa._ffi.lib.cotix_eval
    calls = []

    def checked(*args):
        assert len(args) == len(real.argtypes)
        for t, v in zip(real.argtypes, args):
            if v is not None:
                t.from_param(v)  # raises on a mismatch
        calls.append(args)
        return 0

    monkeypatch.setattr(pa._ffi.lib, "cotix_eval", checked)
    monkeypatch.setattr(torch._C, "_cuda_getCurrentRawStream", lambda i: 0, raising=False)

    class Scen:
        world = _robocup_world_cpu()
        dyn_reset = world.dyn.clone()
        stages = pa._ffi.STAGES_ROBOCUP

    for judge in (None, E.LinearJudge(rate_w={24: 1.0})):
        env = pa.BatchedEnv(Scen(), autoreset=True, judge=judge)
        env.step(1)
        env.step(1)
        assert len(env._launchers) == 1  # one prepared launch for the same configuration
        act = torch.ones(Scen.world.B, 2)
        env.step(1, action=act)
        assert calls[-1][13].value == act.data_ptr() and calls[-2][13] is None
        env.step(4)
        assert len(env._launchers) == 2
        with pytest.raises(ValueError, match="action"):
            env.step(1, action=torch.ones(Scen.world.B, 3))
    assert isinstance(calls[0][-1], ctypes.c_void_p)


def test_tiling_is_a_scene_property():
    """cotix_scene_create picks the default envs per wave from the scene's LDS
    need (4, else the largest of 2 and 1 that fits the CU's 160 KiB with four
    waves per workgroup, else one env per wave in workgroups of 2 or 1 waves)
    and rejects a scene beyond the documented caps, with the reason; an
    explicit tiling that does not fit is rejected by cotix_scene_set_variant."""
    import parallax_amd as pa
    import grad_cases as GC
    import scene_cases
    from test_gpu_parity import _pa_bodies
    quad_row = pa.Scene(_pa_bodies(pa, GC.quad_row_case(1, 1)["make"]()))
    assert quad_row.variant()["envs_per_wave"] == 2 and quad_row.waves_per_group() == 4
    quad_row.set_variant(4)  # an explicit tiling beyond four tiles per CU: workgroups of fewer waves
    assert quad_row.waves_per_group() in (1, 2)
    with pytest.raises(RuntimeError, match="bytes of LDS"):
        pa.Scene(_pa_bodies(pa, scene_cases.octagon_row(15))).set_variant(8)
    quad_row.set_variant(1)
    quad_row.set_variant(0)
    assert quad_row.variant()["envs_per_wave"] == 2
    nine = pa.Scene(_pa_bodies(pa, scene_cases.octagon_row(9)))
    assert nine.variant()["envs_per_wave"] == 1 and nine.waves_per_group() == 4
    # beyond four tiles per CU: one env per wave in workgroups of 2 (or 1) waves
    for bodies in (scene_cases.octagon_row(12), scene_cases.octagon_row(15), scene_cases.polygon20()):
        big = pa.Scene(_pa_bodies(pa, bodies))
        assert big.variant() == {"envs_per_wave": 1, "specialization": "generic"}
        assert big.waves_per_group() in (1, 2)
    # the documented hard caps are rejected at creation with the reason
    with pytest.raises(RuntimeError, match="too many cells"):
        pa.Scene(_pa_bodies(pa, scene_cases.octagon_row(16)))
    assert pa.Scene(pa.scenarios.lunar_lander_bodies(torch.zeros(1, 7, 4, 2))).variant()["envs_per_wave"] == 4
    assert pa.Scene(pa.scenarios.robocup_bodies()).waves_per_group() == 4
