"""Generates tests/golden/broadphase_cases.npz: near-touching polygon pairs
whose world AABBs are separated by a POSITIVE gap (1..63 ulps) but whose
reference contact (polygon_vs_polygon, cotix/_contacts.py:294-315, through
the C port of the oracle) is not NaN -- rounding makes GJK report a
collision and _contact_from_edges find a term.  A broadphase with margin 0
would drop these contacts; the kernel's margin 2^-8 S + 2^-16 keeps them.

  python tests/golden/make_broadphase_cases.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "..", "oracle")]
import bp_cases as C  # noqa: E402

F = np.float32


def touch_pairs(rng, na, nb, n):
    A_, B_ = [], []
    for _ in range(n):
        S = 10.0 ** rng.uniform(-1, 4)
        A = C._convex(rng, na, S * rng.uniform(0.05, 0.4)) + rng.uniform(-S / 2, S / 2, size=2)
        A = A.astype(F).astype(np.float64)
        B = C._convex(rng, nb, S * rng.uniform(0.05, 0.4))
        va, wb = A[np.argmax(A[:, 0])], B[np.argmin(B[:, 0])]
        ulp = float(np.spacing(F(max(abs(va[0]), 1e-30))))
        off = np.array([rng.integers(1, 64) * ulp, rng.integers(-8, 9) * ulp])
        A_.append(A.astype(F))
        B_.append((B - wb + va + off).astype(F))
    return np.array(A_, F), np.array(B_, F)


def main():
    out = {}
    for na, nb, want in ((4, 4, 8), (4, 6, 8)):
        rng = np.random.default_rng(100 * na + nb)
        keepA, keepB = [], []
        while len(keepA) < want:
            A, B = touch_pairs(rng, na, nb, 20000)
            res = C.oracle_contacts(A, B)
            for i in np.nonzero(~np.isnan(res[:, 2]))[0]:
                if C.aabb_gap(A[i], B[i]) > 0 and len(keepA) < want:
                    keepA.append(A[i])
                    keepB.append(B[i])
        out["touch_%d%d_a" % (na, nb)] = np.array(keepA, F)
        out["touch_%d%d_b" % (na, nb)] = np.array(keepB, F)
        print(na, nb, len(keepA))
    np.savez(C.GOLD, **out)


if __name__ == "__main__":
    main()
