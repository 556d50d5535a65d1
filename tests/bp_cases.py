"""Adversarial cases for the polygon broadphase (COTIX_STAGE_BROADPHASE,
DESIGN.md section 3 "Broadphase exactness"), shared by the CPU (host
emulation, mutation builds) and GPU tests.

A case is a pair of WORLD polygons (A: n_a vertices, B: n_b vertices).  The
test scene has two bodies at the origin with angle 0 (static A, dynamic B at
rest), so the kernel's world shapes are these vertices exactly, and one
collider step decides the pair's contact.  Sets:
  touch      near-touching pairs at a positive AABB gap (1..63 ulps) whose
             reference contact is NOT NaN (harvested from the C port of the
             oracle): a broadphase with margin 0 would drop them
  collinear  an edge of A and an edge of B on one line (the configuration in
             which rounding makes _contact_from_edges accept an edge
             intersection across a gap), gaps in [margin, 4 margin]
  sliver     polygons with a sharp vertex near the 0.5 degree limit, gaps in
             [margin, 4 margin]
  far        |coordinates| up to ~1e4, gaps in [margin, 4 margin]
  nonfinite  a NaN or inf vertex coordinate
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..", "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

F = np.float32
GOLD = os.path.join(HERE, "golden", "broadphase_cases.npz")


def margin_of(A, B):
    S = max(np.abs(A).max(), np.abs(B).max())
    return F(F(F(S) * F(0.00390625)) + F(1.52587890625e-05))


def aabb_gap(A, B):
    lo_a, hi_a, lo_b, hi_b = A.min(0), A.max(0), B.min(0), B.max(0)
    return max(F(lo_b[0] - hi_a[0]), F(lo_a[0] - hi_b[0]), F(lo_b[1] - hi_a[1]), F(lo_a[1] - hi_b[1]))


def _convex(rng, n, r, sharp=None):
    if sharp is None:
        ang = np.sort(rng.uniform(-np.pi, np.pi, size=n))
    else:  # one vertex with interior angle ~`sharp` degrees: a thin isosceles spike
        half = np.deg2rad(sharp) / 2
        ang = np.concatenate([[0.0], np.sort(rng.uniform(np.pi - 1.2, np.pi + 1.2, size=n - 1))])
        pts = [(r * 1.0, 0.0)]
        # the spike tip at angle 0, its two neighbours on the rays at +-half from the tip
        base = r * 0.8
        pts.append((r - base * np.cos(half), base * np.sin(half)))
        pts.append((r - base * np.cos(half), -base * np.sin(half)))
        rest = [(-r * 0.3 * np.cos(a), r * 0.3 * np.sin(a)) for a in np.linspace(-0.5, 0.5, n - 3)] if n > 3 else []
        P = np.array(pts + rest)
        return P
    rad = r * rng.uniform(0.5, 1.0, size=n)
    return np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)


def _place_right(rng, A, B, gap):
    """B shifted so that its AABB starts `gap` right of A's (+ random y)."""
    B = B - [B[:, 0].min(), 0] + [A[:, 0].max() + gap, rng.uniform(-0.5, 0.5) * np.ptp(A[:, 1])]
    return B


def gen_set(name, na, nb, n, seed):
    """n pairs (A [n, na, 2], B [n, nb, 2]) f32 world vertices of a set."""
    from bp_adversarial import convex_on_line
    rng = np.random.default_rng(seed)
    As, Bs = [], []
    while len(As) < n:
        S = 10.0 ** rng.uniform(-1, 2) if name != "far" else 10.0 ** rng.uniform(3, 4)
        if name == "collinear":
            L = S * rng.uniform(0.05, 0.4)
            A = convex_on_line(rng, na, -L, 0.0, True)
            B0 = convex_on_line(rng, nb, 0.0, S * rng.uniform(0.05, 0.4), bool(rng.integers(2)))
            th = rng.uniform(-np.pi, np.pi)
            R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
            T = rng.uniform(-S, S, size=2)
            A = (A @ R.T + T).astype(F).astype(np.float64)
            # slide B along the shared line until the AABB gap is in [m, 4m]
            d = R @ [1.0, 0.0]
            m = float(margin_of(A.astype(F), (B0 @ R.T + T).astype(F)))
            lo, hi = 0.0, 4 * S
            Bw = None
            for _ in range(60):
                mid = (lo + hi) / 2
                Bt = (B0 @ R.T + T + d * mid).astype(F)
                g = float(aabb_gap(A.astype(F), Bt))
                if g < m:
                    lo = mid
                elif g > 4 * m:
                    hi = mid
                else:
                    Bw = Bt
                    break
            if Bw is None:
                continue
            As.append(A.astype(F))
            Bs.append(Bw)
            continue
        A = _convex(rng, na, S * rng.uniform(0.1, 0.4), sharp=rng.uniform(0.45, 0.7) if name == "sliver" else None)
        A = (A + rng.uniform(-S, S, size=2) * (0.5 if name != "far" else 1.0)).astype(F).astype(np.float64)
        B0 = _convex(rng, nb, S * rng.uniform(0.1, 0.4))
        B0 = B0 - [B0[:, 0].min(), 0] + [A[:, 0].max(), rng.uniform(-0.5, 0.5) * np.ptp(A[:, 1]) + A[:, 1].mean()]
        k = rng.uniform(1.0, 4.0)
        lo, hi, B = 0.0, 2 * S, None
        for _ in range(80):  # shift B right until the gap / margin ratio is ~k
            mid = (lo + hi) / 2
            Bt = (B0 + [mid, 0.0]).astype(F)
            r = float(aabb_gap(A.astype(F), Bt)) / float(margin_of(A.astype(F), Bt))
            if r < k:
                lo = mid
            else:
                hi, B = mid, Bt
            if B is not None and abs(r - k) < 0.05:
                break
        if B is None:
            continue
        A = A.astype(F)
        if rng.random() < 0.5:  # the gap along y instead
            A, B = A[:, ::-1].copy(), B[:, ::-1].copy()
        if name == "nonfinite":
            k = rng.integers(na if rng.random() < 0.5 else nb)
            bad = [np.nan, np.inf, -np.inf][rng.integers(3)]
            (A if k < na and rng.random() < 0.5 else B)[k % min(na, nb), rng.integers(2)] = bad
        As.append(np.ascontiguousarray(A, F))
        Bs.append(np.ascontiguousarray(B, F))
    return np.array(As, F), np.array(Bs, F)


def load_touch():
    g = np.load(GOLD)
    return {k: g[k] for k in g.files}


def oracle_contacts(A, B):
    """(pen, cp) [n, 4] of polygon_vs_polygon on sorted copies, C port."""
    from cotix_oracle import cport
    from cotix_oracle import geometry as G
    lib = cport.load()
    n, na, nb = A.shape[0], A.shape[1], B.shape[1]
    ra, rb = np.zeros((n, 18), F), np.zeros((n, 18), F)
    for i in range(n):
        for rows, V, nv in ((ra, A[i], na), (rb, B[i], nb)):
            vs = G.order_clockwise([tuple(v) for v in V])
            rows[i, 0], rows[i, 1] = 2, nv
            rows[i, 2:2 + 2 * nv] = np.array(vs, F).reshape(-1)
    out = np.zeros((n, 4), F)
    P = ctypes.c_void_p
    lib.oracle_contacts(3, n, ra.ctypes.data_as(P), rb.ctypes.data_as(P), out.ctypes.data_as(P), None)
    return out


def scene_bodies(na, nb):
    """Oracle bodies of the two-body test scene (geometry per env)."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    inf = float("inf")
    a = P.Body([G.Polygon([(0, 0), (1, 0), (1, 1), (0, 1), (0.5, 1.5), (-0.5, 0.5)][:na], kind="Polygon%d" % na)],
               mass=inf, inertia=inf)
    b = P.Body([G.Polygon([(0, 0), (1, 0), (1, 1), (0, 1), (0.5, 1.5), (-0.5, 0.5)][:nb], kind="Polygon%d" % nb)],
               mass=1.0, inertia=1.0)
    return [a, b]


def geometry_rows(A, B):
    """Per-env local geometry rows (sorted vertices, as Polygon.__init__)."""
    from cotix_oracle import geometry as G
    rows = []
    for a, b in zip(A, B):
        ra = np.array(G.order_clockwise([tuple(v) for v in a]), F).reshape(-1)
        rb = np.array(G.order_clockwise([tuple(v) for v in b]), F).reshape(-1)
        rows.append(np.concatenate([ra, rb]))
    return np.ascontiguousarray(np.stack(rows), F)
