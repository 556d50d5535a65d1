"""The C port of the oracle (bench's CPU baseline and fast checker) must
reproduce the Python oracle's golden traces -- state, keys, error bits and
the collider's contact choices (chosen partner per body, winning candidate
per cell) -- and contact fixtures bit for bit."""
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def cp():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "..", "oracle")], check=True)
    from cotix_oracle import cport
    return cport, cport.load()


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _trace(sc, tr, stages, geom=None):
    dyn = np.ascontiguousarray(tr["dyn"][0].transpose(1, 2, 0))
    keys = np.ascontiguousarray(tr["keys"][0]).astype(np.uint32)
    err = np.zeros(dyn.shape[2], np.uint32)
    for t in range(tr["err"].shape[0]):
        ch, cl = sc.step_ex(dyn, keys, err, 1, stages, geom, trace=True, nthreads=2)
        assert np.array_equal(ch[0].T, tr["chosen"][t]), "chosen step %d" % t
        assert np.array_equal(cl[0].transpose(2, 0, 1), tr["cells"][t]), "cells step %d" % t
        assert same_f32(dyn.transpose(2, 0, 1), tr["dyn"][t + 1]), "step %d" % t
        assert np.array_equal(keys, tr["keys"][t + 1])
        assert np.array_equal(err, np.bitwise_or.reduce(tr["err"][: t + 1], axis=0))


def test_cport_robocup(cp):
    cport, lib = cp
    from cotix_oracle import physics as P
    _trace(cport.Scene(lib, P.robocup_bodies()), np.load(os.path.join(GOLD, "robocup_trace.npz")),
           cport.STAGES_ROBOCUP)


def test_cport_lunar(cp):
    cport, lib = cp
    from cotix_oracle import physics as P
    tr = np.load(os.path.join(GOLD, "lunar_trace.npz"))
    rows = np.stack([cport.Scene(lib, P.lunar_lander_bodies(k)).geom for k in tr["terrain_keys"]])
    _trace(cport.Scene(lib, P.lunar_lander_bodies(tr["terrain_keys"][0])), tr, cport.STAGES_LUNAR, rows)


def test_cport_box_world(cp):
    cport, lib = cp
    import sys
    sys.path.insert(0, GOLD)
    import make_golden as mg
    tr = np.load(os.path.join(GOLD, "box_world_trace.npz"))
    for e in range(tr["dyn"].shape[1]):
        sub = {k: tr[k][:, e:e + 1] for k in ("dyn", "keys", "err", "chosen", "cells")}
        _trace(cport.Scene(lib, mg.box_world_bodies(e)), sub, cport.STAGES_ROBOCUP)


@pytest.mark.parametrize("name", ["aabb_aabb", "circle_circle", "circle_aabb", "poly_poly", "aabb_poly",
                                  "circle_poly"])
def test_cport_contacts(cp, name):
    cport, lib = cp
    g = np.load(os.path.join(GOLD, "contacts.npz"))
    a, b = np.ascontiguousarray(g[name + "_a"]), np.ascontiguousarray(g[name + "_b"])
    out = np.zeros((a.shape[0], 4), np.float32)
    err = np.zeros(a.shape[0], np.uint32)
    lib.oracle_contacts(int(g[name + "_fn"]), a.shape[0], cport._p(a), cport._p(b), cport._p(out), cport._p(err))
    assert same_f32(out, g[name + "_out"])
    assert np.array_equal(err, g[name + "_err"].astype(np.uint32))
