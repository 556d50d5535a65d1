"""TEST INFRASTRUCTURE ONLY -- scalar restatement of the reference's design by
contract (cotix/_design_by_contract.py:13-107) for one env at a time, the
checker of parallax_amd.contracts and of the device state check
(cotix_check_state).

The reference wraps eqx.error_if; with EQX_ON_ERROR=nan (the build's mode,
DESIGN.md section 4) a tripped condition turns every float leaf of the guarded
value into NaN.  Per env of a batch that is: the env's guarded floats become
NaN and, for a world state, its error word gets ERR_CONTRACT.  The state
invariant the device checks is the one the reference's invariant message
names ("Probably nan or invalid value encountered in the checked class",
:87-91): a NaN or infinite state word.  Plain Python / numpy loops, one env
per call.
"""
import math

import numpy as np

ERR_CONTRACT = 8
ERR_STATE_NONFINITE = 4


def error_if(value, pred):
    """eqx.error_if(value, pred) under EQX_ON_ERROR=nan for ONE env: value is
    a float, a list/tuple of values, or a dict; every float becomes NaN when
    pred holds (:20-25, :41-51, :84-90)."""
    if not pred:
        return value
    if isinstance(value, np.floating):
        return type(value)(math.nan)
    if isinstance(value, float):
        return math.nan
    if isinstance(value, (list, tuple)):
        return type(value)(error_if(v, True) for v in value)
    if isinstance(value, dict):
        return {k: error_if(v, True) for k, v in value.items()}
    return value


def env_state_error_if(dyn_env, err_env, pred):
    """error_if on one env of a world state: (dyn words, err word)."""
    if not pred:
        return list(dyn_env), err_env
    return [math.nan] * len(dyn_env), err_env | ERR_CONTRACT


def pre_condition(condition, func, *args):
    """pre_condition(condition)(func)(*args) for one env (:13-31): the inputs
    are guarded by NOT condition before the call."""
    bad = not condition(*args)
    return func(*error_if(list(args), bad))


def post_condition(condition, func, *args, provide_input=False):
    """post_condition(condition, provide_input)(func)(*args) (:34-57)."""
    r = func(*args)
    ok = condition(r, *args) if provide_input else condition(r)
    return error_if(r, not ok)


def class_invariant_fires(invariant_value):
    """_check_invariant (:71-91): the invariant's value IS eqx.error_if's
    condition -- the guard fires where __invariant__() is true."""
    return bool(invariant_value)


def state_nonfinite(dyn_env):
    """The device state invariant: some state word is NaN or +-inf."""
    return any(not math.isfinite(float(v)) for v in dyn_env)


def check_state(dyn, err):
    """cotix_check_state's contract on a batch: dyn [n_bodies][6][B], err [B];
    err[e] |= ERR_STATE_NONFINITE for every env whose state fails the
    invariant (env by env, scalar)."""
    dyn = np.asarray(dyn, np.float32)
    out = np.array(err, np.int64, copy=True)
    for e in range(dyn.shape[2]):
        if state_nonfinite(dyn[:, :, e].reshape(-1).tolist()):
            out[e] |= ERR_STATE_NONFINITE
    return out
