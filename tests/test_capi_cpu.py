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
