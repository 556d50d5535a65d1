"""Kernel-logic parity on CPU: the fused step kernel's phase code
(parallax_amd/csrc/cotix_kernel.h), compiled for the host by the test-only
emulation harness (tests/emu), must reproduce the golden oracle traces bit
for bit -- the same bar as the GPU tests -- for every envs-per-wave tiling."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(HERE, "emu"))
sys.path.insert(0, GOLD)


@pytest.fixture(scope="module")
def emu_lib():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    import emu
    return emu, emu.load()


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def run_trace(emu, lib, bodies, geom_rows, tr, stages, EW, per_env_geom):
    h, geom = emu.oracle_scene(lib, bodies)
    B = tr["dyn"].shape[1]
    T = tr["err"].shape[0]
    if per_env_geom:
        geom = np.ascontiguousarray(np.stack(geom_rows).astype(np.float32))
        gstride = geom.shape[1]
    else:
        gstride = 0
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(np.uint32)
    err = np.zeros(B, np.uint32)
    for t in range(T):
        emu.step(lib, h, dyn, keys, err, geom, gstride, 1, stages, E=EW)
        got = dyn.transpose(2, 0, 1)
        assert same_f32(got, tr["dyn"][t + 1]), "step %d" % t
        assert np.array_equal(keys, tr["keys"][t + 1]), "keys step %d" % t
        assert np.array_equal(err, np.bitwise_or.reduce(tr["err"][: t + 1], axis=0)), "err step %d" % t


@pytest.mark.parametrize("EW", [1, 2, 4])
def test_emu_robocup_trace(emu_lib, EW):
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "robocup_trace.npz"))
    run_trace(emu, lib, P.robocup_bodies(), None, tr, 1 | 4 | 16, EW, False)


@pytest.mark.parametrize("EW", [1, 2, 4])
def test_emu_lunar_trace(emu_lib, EW):
    emu, lib = emu_lib
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    rows = []
    for k in tr["terrain_keys"]:
        _, g = emu.oracle_scene(lib, P.lunar_lander_bodies(k))
        rows.append(g)
    run_trace(emu, lib, P.lunar_lander_bodies(tr["terrain_keys"][0]), rows, tr, 1 | 2 | 4 | 8 | 16, EW, True)


def test_emu_box_world_trace(emu_lib):
    emu, lib = emu_lib
    import make_golden as mg
    tr = np.load(os.path.join(GOLD, "box_world_trace.npz"))
    for e in range(tr["dyn"].shape[1]):
        sub = {k: tr[k][:, e:e + 1] for k in ("dyn", "keys", "err")}
        run_trace(emu, lib, mg.box_world_bodies(e), None, sub, 1 | 4 | 16, 2, False)


def test_emu_order_clockwise_ties_nan_zero(emu_lib):
    """Stable order by angle (the kernel's rank sort) == the oracle's
    insertion sort, on duplicate vertices (ties), NaN coordinates and
    vertices whose angle is +-0 / +-pi."""
    emu, lib = emu_lib
    from cotix_oracle import geometry as G
    rng = np.random.default_rng(4)
    cases = []
    for nv in (3, 4, 6, 8):
        for _ in range(200):
            xy = rng.integers(-2, 3, size=(nv, 2)).astype(np.float32)  # many duplicates / collinear
            if rng.random() < 0.2:
                xy[rng.integers(nv), rng.integers(2)] = np.nan
            if rng.random() < 0.2:
                xy[rng.integers(nv)] = (-0.0, 0.0)
            cases.append(xy)
    for xy in cases:
        nv = xy.shape[0]
        got = np.ascontiguousarray(xy.reshape(-1).copy())
        lib.emu_order_clockwise(got.ctypes.data_as(emu.P_), 1, nv)
        want = np.array(G.order_clockwise([tuple(v) for v in xy]), np.float32).reshape(-1)
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (xy, got.reshape(-1, 2), want.reshape(-1, 2))
