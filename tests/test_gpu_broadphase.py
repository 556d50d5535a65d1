"""The polygon broadphase on the GPU: the adversarial sets of
tests/bp_cases.py (near-touching witnesses whose reference contact is not
NaN at a positive gap, collinear edges, slivers at the 0.5 degree limit,
|coordinates| ~1e4, NaN / inf vertices) through the step kernel with the
broadphase on and off, against the C port of the oracle -- state, keys, err
and the collider trace bit for bit."""
import numpy as np
import pytest

import bp_cases as C

pytestmark = pytest.mark.gpu
F = np.float32


def _sets():
    g = C.load_touch()
    yield "touch44", g["touch_44_a"], g["touch_44_b"]
    yield "touch46", g["touch_46_a"], g["touch_46_b"]
    for k, name in enumerate(("collinear", "sliver", "far", "nonfinite")):
        for na, nb in ((4, 4), (4, 6)):
            A, B = C.gen_set(name, na, nb, 48, 10 * k + nb)
            yield "%s%d%d" % (name, na, nb), A, B


@pytest.mark.parametrize("name,A,B", list(_sets()), ids=lambda x: x if isinstance(x, str) else "")
def test_broadphase_gpu_vs_cport(name, A, B):
    import torch
    assert torch.cuda.is_available()
    import parallax_amd as pa
    from test_broadphase_cpu import run_cport, same
    na, nb, n = A.shape[1], B.shape[1], A.shape[0]
    rows = C.geometry_rows(A, B)
    P = {4: pa.Polygon4, 6: pa.Polygon6}
    ga = torch.tensor(rows[:, :2 * na].reshape(n, na, 2))
    gb = torch.tensor(rows[:, 2 * na:].reshape(n, nb, 2))
    inf = float("inf")
    bodies = [pa.AnyBody(shape=pa.UniversalShape(P[na](ga, presorted=True)), mass=inf, inertia=inf),
              pa.AnyBody(shape=pa.UniversalShape(P[nb](gb, presorted=True)), mass=1.0, inertia=1.0)]
    keys = torch.tensor(np.stack([np.arange(n), np.arange(n) * 7 + 1], 1).astype(np.uint32).view(np.int32))
    want = run_cport(A, B)
    for bp in (pa._ffi.STAGE_BROADPHASE, 0):
        w = pa.World(bodies, n, "cuda", keys.clone())
        w.dyn.zero_()
        tr = {}
        w.step(1, 1e-2, pa._ffi.STAGES_ROBOCUP | bp, trace=tr)
        torch.cuda.synchronize()
        assert same(w.dyn.cpu().numpy(), want[0]), (name, bp)
        assert np.array_equal(w.keys.cpu().numpy().view(np.uint32), want[1]), (name, bp)
        assert np.array_equal(w.err.cpu().numpy().view(np.uint32), want[2]), (name, bp)
        assert np.array_equal(tr["chosen"].cpu().numpy(), want[3]), (name, bp)
        assert np.array_equal(tr["cells"].cpu().numpy(), want[4]), (name, bp)
