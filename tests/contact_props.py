"""Port of the reference's contact invariants ``_test_contact_info``
(test/test_collisions.py:75-159) over any contact function f(a, b) ->
(pen, cp) with shapes exposing move()/contains().  Shared by the oracle tests
(CPU) and the HIP operator tests (GPU)."""
import numpy as np

F = np.float32


def _norm(v):
    return float(np.sqrt(np.float64(v[0]) ** 2 + np.float64(v[1]) ** 2))


def check_contact_info(f, a, b, heavy=True, small_eps=1e-5):
    big_eps = 10 * small_eps
    pen, cp = f(a, b)
    if np.isnan(cp[0]) or np.isnan(cp[1]):
        return True
    contained = a.contains(cp) and b.contains(cp)
    an = a.move(pen)
    pen2, _ = f(an, b)
    after_ok = _norm(pen2) < small_eps
    no_shorter = True
    deep = True
    if heavy:
        ang = np.linspace(0, 2 * np.pi, 20).astype(F)
        length = max(_norm(pen) - big_eps, 0.0)
        ok = []
        for t in ang:
            d = (F(np.cos(t) * length), F(np.sin(t) * length))
            p3, _ = f(a.move(d), b)
            ok.append(_norm(p3) > small_eps)
        no_shorter = all(ok) or (_norm(pen) < 1.5 * small_eps)
        dd = []
        for t in ang:
            d = (F(np.cos(t) * big_eps), F(np.sin(t) * big_eps))
            p4, _ = f(an.move(d), b)
            dd.append(_norm(p4) > big_eps * 0.5)
        deep = any(dd)
    return bool(deep and after_ok and no_shorter and contained)
