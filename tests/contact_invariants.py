"""Batched port of the reference's contact invariants ``_test_contact_info``
(test/test_collisions.py:75-159) for the HIP operator kernels: every case of
a batch is checked at once on the device, f(a, b) being ``cotix_contacts``
over [n, 18] shape rows (kind, nverts, d[16]; parallax_amd.run_contacts).
TEST INFRASTRUCTURE ONLY.  Arithmetic follows tests/contact_props.py (the
scalar port used on the CPU oracle) so that both give the same per-case
verdict: moves, containment and the probe vectors in f32, norms in f64 --
see test_gpu_invariants.py, which compares them case by
case on a sample.

The reference's ``same_edging`` term (:92-100) calls
``_contact_from_edges(edges_a, edges_b)`` with two of its six arguments and
therefore cannot run for the polygon/AABB pairs it is meant for (the
reference skips those tests as "not implemented"); it is left out here.
"""
import numpy as np
import torch

F32 = torch.float32
N_DIRS = 20


def _norm64(v):
    v = v.double()
    return torch.sqrt(v[..., 0] ** 2 + v[..., 1] ** 2)


def _sort_polys(rows):
    """Polygon.__init__ re-sorts the vertices (cotix/_convex_shapes.py:143-144):
    cotix_order_clockwise on the rows' vertex block (one vertex count per batch)."""
    import parallax_amd as pa
    nv = int(rows[0, 1].item())
    v = rows[:, 2:2 + 2 * nv].contiguous()
    pa._ffi.check(pa._ffi.lib.cotix_order_clockwise(pa._ffi.ptr(v), v.shape[0], nv, pa._ffi.stream_ptr(v.device)),
                  "cotix_order_clockwise")
    out = rows.clone()
    out[:, 2:2 + 2 * nv] = v
    return out


def move(rows, delta):
    """shape.move(delta) (cotix/_convex_shapes.py:34-35,108-111,177-179) for a
    batch of one kind; delta f32 [n, 2]."""
    kind = int(rows[0, 0].item())
    out = rows.clone()
    if kind == 0:  # circle (r, cx, cy)
        out[:, 3:5] = rows[:, 3:5] + delta
    elif kind == 1:  # AABB (lo, up)
        out[:, 2:4] = rows[:, 2:4] + delta
        out[:, 4:6] = rows[:, 4:6] + delta
    else:
        nv = int(rows[0, 1].item())
        for k in range(nv):
            out[:, 2 + 2 * k:4 + 2 * k] = rows[:, 2 + 2 * k:4 + 2 * k] + delta
        out = _sort_polys(out)
    return out


def contains(rows, p):
    """shape.contains(p) (cotix/_convex_shapes.py:28-29,105-106,168-175), f32."""
    kind = int(rows[0, 0].item())
    eps = torch.tensor(1e-6, dtype=F32, device=rows.device)
    if kind == 0:
        d = p - rows[:, 3:5]
        return (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) <= (rows[:, 2] + eps) * (rows[:, 2] + eps)
    if kind == 1:
        lo, up = rows[:, 2:4], rows[:, 4:6]
        return ((p >= lo - eps) & (p <= up + eps)).all(-1)
    nv = int(rows[0, 1].item())
    vs = rows[:, 2:2 + 2 * nv].reshape(-1, nv, 2)
    e0, e1 = vs, torch.roll(vs, 1, dims=1)  # edge k = (v_k, v_{k-1})
    d = e0 - e1
    q = p[:, None, :] - e0
    dots = q[..., 0] * (-d[..., 1]) + q[..., 1] * d[..., 0]
    s = torch.sign(dots)
    return (s == s[:, :1]).all(-1)


def check(f, a, b, heavy, small_eps=1e-5):
    """Per-case verdict (bool [n]) of _test_contact_info(f, a, b, heavy)."""
    big = 10 * small_eps
    pen, cp = f(a, b)
    nan = torch.isnan(cp).any(-1)
    ok = contains(a, cp) & contains(b, cp)
    an = move(a, pen)
    pen2, _ = f(an, b)
    ok &= _norm64(pen2) < small_eps
    if heavy:
        # directions: f32 linspace, f32 cos/sin (numpy's, as contact_props), f32 products
        ang = np.linspace(0, 2 * np.pi, N_DIRS).astype(np.float32)
        npen = _norm64(pen)
        length = torch.clamp(npen - big, min=0.0).to(F32)
        bigf = np.float32(big)
        shorter = torch.ones_like(ok)
        deep = torch.zeros_like(ok)
        for t in ang:
            cs = torch.tensor([np.cos(t), np.sin(t)], dtype=F32, device=a.device)
            d = length[:, None] * cs[None, :]
            p3, _ = f(move(a, d), b)
            shorter &= _norm64(p3) > small_eps
            d2 = torch.tensor([np.cos(t) * bigf, np.sin(t) * bigf], dtype=F32, device=a.device)
            p4, _ = f(move(an, d2.expand(a.shape[0], 2)), b)
            deep |= _norm64(p4) > big * 0.5
        ok &= (shorter | (npen < 1.5 * small_eps)) & deep
    return nan | ok


# random shapes at the reference's distributions (test/test_collisions.py:186-462)
def rand_circles(n, g, dev):
    r = torch.zeros(n, 18, dtype=F32, device=dev)
    r[:, 2] = torch.rand(n, generator=g, device=dev) * (5.0 - 0.01) + 0.01
    r[:, 3:5] = torch.randn(n, 2, generator=g, device=dev)
    return r


def rand_aabbs(n, g, dev):
    r = torch.zeros(n, 18, dtype=F32, device=dev)
    r[:, 0] = 1
    lo = torch.randn(n, 2, generator=g, device=dev)
    r[:, 2:4] = lo
    r[:, 4:6] = lo + (torch.rand(n, 2, generator=g, device=dev) * (5.0 - 0.01) + 0.01)
    return r


def fixed_polys(n, verts, dev):
    v = torch.tensor(np.asarray(verts, np.float32), device=dev).reshape(-1)
    r = torch.zeros(n, 18, dtype=F32, device=dev)
    r[:, 0], r[:, 1] = 2, len(verts)
    r[:, 2:2 + v.numel()] = v
    return _sort_polys(r)


def rand_polys(n, nv, g, dev):
    r = torch.zeros(n, 18, dtype=F32, device=dev)
    r[:, 0], r[:, 1] = 2, nv
    r[:, 2:2 + 2 * nv] = torch.randn(n, 2 * nv, generator=g, device=dev)
    return _sort_polys(r)


def to_oracle(row):
    """One row -> the oracle's shape object (for per-case comparison)."""
    from cotix_oracle import geometry as G
    row = np.asarray(row, np.float32)
    if row[0] == 0:
        return G.Circle(row[2], (row[3], row[4]))
    if row[0] == 1:
        return G.AABB((row[2], row[3]), (row[4], row[5]))
    nv = int(row[1])
    return G.Polygon([(row[2 + 2 * k], row[3 + 2 * k]) for k in range(nv)], kind="Polygon%d" % nv, sort=False)
