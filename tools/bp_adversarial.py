"""Adversarial search for the polygon broadphase (COTIX_STAGE_BROADPHASE):
pairs whose world AABBs are separated by more than the margin 2^-8 S + 2^-16
but whose reference contact (GJK exists AND _contact_from_edges cp) is not
NaN.  Generates pairs with an edge of A and an edge of B on one line (the
configuration in which rounding makes _contact_from_edges accept an edge
intersection across a gap, and the Minkowski difference has an edge on a line
through the origin), rotated and translated to f32 world coordinates, and
runs them through the C port of the oracle (oracle/build/libcotix_oracle.so).

  python tools/bp_adversarial.py [n_pairs] [seed] [collinear|touch]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from cotix_oracle import cport  # noqa: E402

F = np.float32


def convex_on_line(rng, n, x0, x1, up):
    """n-gon with the edge (x0,0)-(x1,0) and the rest on one side (y > 0 if up)."""
    ang = np.sort(rng.uniform(0.15, np.pi - 0.15, size=n - 2))[::-1]
    cx, w = (x0 + x1) / 2, (x1 - x0) / 2
    h = rng.uniform(0.3, 2.0) * w
    pts = [(x0, 0.0), (x1, 0.0)] + [(cx + w * np.cos(a), h * np.sin(a)) for a in ang]
    pts = np.array(pts)
    if not up:
        pts[:, 1] = -pts[:, 1]
    return pts


def sort_cw(v):
    """order_clockwise's order (ascending atan2 about the mean), f64 keys."""
    m = v.mean(0)
    k = np.arctan2(v[:, 1] - m[1], v[:, 0] - m[0])
    return v[np.argsort(k, kind="stable")]


def random_convex(rng, n, r):
    ang = np.sort(rng.uniform(-np.pi, np.pi, size=n))
    rad = r * rng.uniform(0.5, 1.0, size=n)
    return np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)


def make_touch_pairs(rng, N):
    """A's rightmost vertex and B's leftmost vertex k ulps apart in x (the
    AABB gap), within a few ulps in y: near-touching pairs whose reference
    contact can be non-NaN at a positive gap far below the margin."""
    rows_a = np.zeros((N, 18), F)
    rows_b = np.zeros((N, 18), F)
    gaps = np.zeros(N, F)
    margins = np.zeros(N, F)
    for i in range(N):
        na, nb = rng.integers(3, 7, size=2)
        S = 10.0 ** rng.uniform(-1, 4)
        A = random_convex(rng, na, S * rng.uniform(0.05, 0.4)) + rng.uniform(-S / 2, S / 2, size=2)
        Bv = random_convex(rng, nb, S * rng.uniform(0.05, 0.4))
        A = A.astype(F).astype(np.float64)
        va = A[np.argmax(A[:, 0])]
        wb = Bv[np.argmin(Bv[:, 0])]
        ulp = float(np.spacing(F(max(abs(va[0]), 1e-30))))
        off = np.array([rng.integers(1, 64) * ulp, rng.integers(-8, 9) * ulp])
        Bw = (Bv - wb + va + off).astype(F)
        Aw = A.astype(F)
        Aw, Bw = sort_cw(Aw.astype(np.float64)).astype(F), sort_cw(Bw.astype(np.float64)).astype(F)
        lo_a, hi_a, lo_b, hi_b = Aw.min(0), Aw.max(0), Bw.min(0), Bw.max(0)
        Sx = max(np.abs(Aw).max(), np.abs(Bw).max())
        gaps[i] = max(F(lo_b[0] - hi_a[0]), F(lo_a[0] - hi_b[0]), F(lo_b[1] - hi_a[1]), F(lo_a[1] - hi_b[1]))
        margins[i] = F(F(Sx) * F(0.00390625)) + F(1.52587890625e-05)
        for rows, V in ((rows_a, Aw), (rows_b, Bw)):
            rows[i, 0] = 2
            rows[i, 1] = len(V)
            rows[i, 2:2 + 2 * len(V)] = V.reshape(-1)
    return rows_a, rows_b, gaps, margins


def make_pairs(rng, N):
    rows_a = np.zeros((N, 18), F)
    rows_b = np.zeros((N, 18), F)
    gaps = np.zeros(N, F)
    margins = np.zeros(N, F)
    for i in range(N):
        na, nb = rng.integers(3, 7, size=2)
        S = 10.0 ** rng.uniform(-1, 4)
        L = S * rng.uniform(0.02, 0.4)
        A = convex_on_line(rng, na, -L, 0.0, True)
        g = L * 10.0 ** rng.uniform(-6, 0)  # gap along the shared line
        Lb = S * rng.uniform(0.02, 0.4)
        Bv = convex_on_line(rng, nb, g, g + Lb, bool(rng.integers(2)))
        th = rng.uniform(-np.pi, np.pi) if rng.random() < 0.8 else rng.choice([0, np.pi / 2, np.pi / 4, np.pi])
        c, s = np.cos(th), np.sin(th)
        R = np.array([[c, -s], [s, c]])
        T = rng.uniform(-S, S, size=2)
        Aw = (A @ R.T + T).astype(F)
        Bw = (Bv @ R.T + T).astype(F)
        Aw, Bw = sort_cw(Aw.astype(np.float64)).astype(F), sort_cw(Bw.astype(np.float64)).astype(F)
        if rng.random() < 0.5:
            Aw, Bw = Bw, Aw
        lo_a, hi_a, lo_b, hi_b = Aw.min(0), Aw.max(0), Bw.min(0), Bw.max(0)
        Sx = max(np.abs(Aw).max(), np.abs(Bw).max())
        gap = max(F(lo_b[0] - hi_a[0]), F(lo_a[0] - hi_b[0]), F(lo_b[1] - hi_a[1]), F(lo_a[1] - hi_b[1]))
        gaps[i], margins[i] = gap, F(F(Sx) * F(0.00390625)) + F(1.52587890625e-05)
        for rows, V in ((rows_a, Aw), (rows_b, Bw)):
            rows[i, 0] = 2
            rows[i, 1] = len(V)
            rows[i, 2:2 + 2 * len(V)] = V.reshape(-1)
    return rows_a, rows_b, gaps, margins


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    mode = sys.argv[3] if len(sys.argv) > 3 else "collinear"
    lib = cport.load()
    rng = np.random.default_rng(seed)
    tot = {"pairs": 0, "skipped_by_bp": 0, "skipped_nonnan": 0, "near_nonnan": 0, "near": 0}
    done = 0
    while done < N:
        n = min(20000, N - done)
        a, b, gaps, margins = (make_touch_pairs if mode == "touch" else make_pairs)(rng, n)
        out = np.zeros((n, 4), F)
        err = np.zeros(n, np.uint32)
        P = ctypes.c_void_p
        lib.oracle_contacts(3, n, a.ctypes.data_as(P), b.ctypes.data_as(P), out.ctypes.data_as(P),
                            err.ctypes.data_as(P))
        nonnan = ~np.isnan(out[:, 2])
        skip = gaps > margins
        near = (gaps > 0) & ~skip
        tot["pairs"] += n
        tot["skipped_by_bp"] += int(skip.sum())
        tot["skipped_nonnan"] += int((skip & nonnan).sum())
        tot["near"] += int(near.sum())
        tot["near_nonnan"] += int((near & nonnan).sum())
        for i in np.nonzero(skip & nonnan)[0][:5]:
            print("COUNTEREXAMPLE", gaps[i], margins[i], a[i].tolist(), b[i].tolist(), out[i].tolist(), flush=True)
        done += n
    print(tot)


if __name__ == "__main__":
    main()
