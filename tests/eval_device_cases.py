"""Device judge / control cases for the fused eval (cotix_eval) tests: each
case is a parallax_amd.envs.LinearJudge / AffineControl pair (kernel + torch
side) and its oracle restatement (oracle/cotix_oracle/envs.py), built from
the same numbers."""
import numpy as np

import grad_cases as GC
from cotix_oracle import envs as OE

INF = float("inf")
K = 0.05


def _free():
    return [-INF] * 6, [INF] * 6


def _region(body, **bounds):
    """bounds word=(lo, hi) over px, py, vx, vy, angle, w."""
    lo, hi = _free()
    names = ("px", "py", "vx", "vy", "angle", "w")
    for k, (a, b) in bounds.items():
        q = names.index(k)
        lo[q], hi[q] = a, b
    return lo, hi


def judges(name, ab):
    """(judge kwargs, control kwargs) of a named case for action body ab."""
    o = 6 * ab
    if name == "x_done":  # tests/eval_cases.XJudge / PDControl as a device pair
        lo, hi = _region(ab, px=(1.2, INF))
        j = dict(rate_w={o: 1.0}, end_w={o + 1: 2.0}, regions=[(ab, lo, hi, 0.0)])
        c = dict(body=ab, gain=[[0, 0, K, 0, 0, 0], [0, 0, 0, K, 0, 0]], target=[[0, 0, 1.0, 0, 0, 0], [0] * 6])
        return j, c
    if name == "multi":  # several terms, two regions with rewards, a biased control
        r0 = _region(ab, px=(1.0, INF), vx=(-INF, 2.5))
        r1 = _region(ab, py=(-INF, -1.2))
        j = dict(rate_w={o: 0.5, o + 2: -0.25, o + 5: 0.125}, end_w={o + 1: 3.0, o + 3: -1.0},
                 regions=[(ab, r0[0], r0[1], 10.0), (ab, r1[0], r1[1], -5.0)])
        c = dict(body=ab, gain=[[0.1, 0, 0.05, 0, 0, 0], [0, 0.2, 0, 0, 0, 0.01]],
                 target=[[0.5, 0, 0.3, 0, 0, 0], [0, -0.2, 0, 0, 0, 1.0]], bias=(0.001, -0.002))
        return j, c
    if name == "goal":  # RoboCup: goals as regions, the error trip as done
        yl = _region(ab, px=(-INF, -4.5), py=(-0.5, 0.5))
        bl = _region(ab, px=(4.5, INF), py=(-0.5, 0.5))
        j = dict(rate_w={o + 2: 0.1}, regions=[(ab, yl[0], yl[1], -1.0), (ab, bl[0], bl[1], 1.0)], done_on_error=True)
        c = dict(body=ab, gain=[[0, 0, 0.1, 0, 0, 0], [0, 0, 0, 0.1, 0, 0]], target=[[0, 0, 2.0, 0, 0, 0], [0] * 6])
        return j, c
    if name == "piecewise":  # a piecewise-linear reward rate over rate regions and a saturating control
        r0 = _region(ab, px=(1.2, INF))
        q0 = _region(ab, px=(-INF, 0.0))
        q1 = _region(ab, vx=(0.0, INF), vy=(-INF, 0.2))
        j = dict(rate_w={o: 0.5}, end_w={o + 1: 1.0}, regions=[(ab, r0[0], r0[1], 2.0)],
                 rate_regions=[(ab, q0[0], q0[1], {o + 2: -2.0, o + 5: 0.25}, 1.5), (ab, q1[0], q1[1], {}, -0.75)])
        c = dict(body=ab, gain=[[0.4, 0, 0.3, 0, 0, 0], [0, 0.5, 0, 0.2, 0, 0]],
                 target=[[0.0, 0, 1.5, 0, 0, 0], [0, 0.5, 0, 0, 0, 0]], bias=(0.01, 0.0),
                 clip=((-0.02, 0.03), (-0.05, 0.01)))
        return j, c
    raise KeyError(name)


def device(name, ab):
    from parallax_amd import envs as E
    j, c = judges(name, ab)
    return E.LinearJudge(**j), E.AffineControl(**c)


def oracle(name, ab):
    j, c = judges(name, ab)
    return OE.LinearJudge(**j), OE.AffineControl(**c)


def case(scene, B, seed=0):
    """(grad_cases case dict, judge name) for a scene."""
    if scene == "box":
        c = GC.box_case(B, 1, seed=seed)
        c["S0"][1, c["ab"], 0] = 1.5  # env 1 done before the first NFE (x_done / multi)
        return c
    return GC.robocup_case(B, 1, seed=seed)


def oracle_eval(case_, name, nfe, wfe, period, with_err=True):
    """Per env: ((bodies, key[, err]), reward, finished) of the oracle's
    restatement of the reference eval with the oracle judge / control."""
    ab = case_["ab"]
    oj, oc = oracle(name, ab)
    out = []
    B = case_["S0"].shape[0]
    for e in range(B):
        bodies = case_["make"]()
        for b, row in zip(bodies, case_["S0"][e]):
            b.set_dyn(row)
        st = (bodies, np.asarray(case_["keys"][e], np.uint32)) + ((0,) if with_err else ())
        out.append(OE.eval_env(case_["step"], st, oc, oj, period, nfe, wfe, GC.D0, ab, carry=(0.0, False)))
    return out
