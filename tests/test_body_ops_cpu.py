"""Body-level UniversalShape operators (cotix/_universal_shape.py:87-132):
collides_with / penetrates_with (GJK over part pairs + EPA-48 through the
reference's wrap_local_support) and the AABB broadphase, in the kernels'
device code compiled for the host, against the oracle bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

import body_cases as BC
import grad_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    sys.path.insert(0, os.path.join(HERE, "emu"))
    import emu
    return emu, emu.load()


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return bool(((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all())


@pytest.mark.parametrize("pair", [(0, 1), (1, 2), (2, 0), (1, 1)])
def test_penetrates_with_matches_oracle(emu_lib, pair):
    emu, lib = emu_lib
    from cotix_oracle import universal as U
    B = 200
    make = lambda: BC.bodies(3)  # noqa: E731
    h, geom = emu.oracle_scene(lib, make())
    dyn = BC.states(B, seed=7)
    col = np.zeros(B, np.int32)
    pen = np.zeros((B, 2), np.float32)
    P = emu.P_
    assert lib.emu_body_penetration(h, dyn.ctypes.data_as(P), geom.ctypes.data_as(P), 0, B, pair[0], pair[1],
                                    col.ctypes.data_as(P), pen.ctypes.data_as(P)) == 0
    hits = 0
    for e in range(B):
        ok, p = U.penetrates_with(BC.oracle_body(make, dyn, e, pair[0]), BC.oracle_body(make, dyn, e, pair[1]), GC.D0)
        assert bool(col[e]) == ok, e
        assert same(pen[e], np.array(p, np.float32)), (e, pen[e], p)
        hits += ok
    assert 0 < hits < B or pair[0] == pair[1]


def test_body_aabb_matches_oracle(emu_lib):
    emu, lib = emu_lib
    from cotix_oracle import universal as U
    B = 200
    make = lambda: BC.bodies(3)  # noqa: E731
    h, geom = emu.oracle_scene(lib, make())
    dyn = BC.states(B, seed=9)
    P = emu.P_
    for b in range(3):
        out = np.zeros((B, 4), np.float32)
        err = np.zeros(B, np.uint32)
        assert lib.emu_body_aabb(h, dyn.ctypes.data_as(P), geom.ctypes.data_as(P), 0, B, b, out.ctypes.data_as(P),
                                 err.ctypes.data_as(P)) == 0
        for e in range(B):
            box, er = U.body_aabb(BC.oracle_body(make, dyn, e, b))
            assert same(out[e], np.array(box, np.float32)), (b, e, out[e], box)
            assert err[e] == er
