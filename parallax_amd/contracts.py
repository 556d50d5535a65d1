"""Design by contract for the batched world (cotix/_design_by_contract.py).

The reference wraps eqx.error_if: a failing condition raises (or, under
EQX_ON_ERROR=nan, turns the guarded values into NaN).  On a batch of
independent envs a condition is a bool tensor [B] and a failure belongs to
the envs it holds for: those envs' guarded floats become NaN and -- for a
WorldState -- their error word gets ERR_CONTRACT (the same per-env error
bitmask the kernels write; ERR_STATE_NONFINITE comes from the device check
World.check_state / cotix_check_state).  Conditions are torch code; the
device path never routes through here.

  pre_condition(condition)                         :13-31
  post_condition(condition, provide_input=False)   :34-57
  class_invariant(cls)                             :80-107
"""
import functools

import torch

from . import _ffi

ERR_CONTRACT = 8  # pre/post condition or invariant failed (beside the kernels' bits 1, 2, 4)


def _mask(pred, B):
    if isinstance(pred, bool):
        return torch.full((B,), pred, dtype=torch.bool)
    m = torch.as_tensor(pred).to(torch.bool)
    if m.dim() == 0:
        m = m.expand(B)
    return m


def error_if(x, pred, env_dim=0):
    """eqx.error_if(x, pred) with EQX_ON_ERROR=nan, per env: every float
    tensor in x (tensors, WorldState, tuples/lists/dicts of them) is NaN for
    the envs where pred holds; a WorldState's err gets ERR_CONTRACT.  Plain
    tensors carry the env batch on `env_dim`; WorldState.dyn on its last
    dimension (the kernels' SoA layout)."""
    from .envs import WorldState
    if isinstance(x, WorldState):
        m = _mask(pred, x.err.shape[0]).to(x.err.device)
        dyn = torch.where(m, torch.full_like(x.dyn, float("nan")), x.dyn)
        err = torch.where(m, x.err | ERR_CONTRACT, x.err)
        return WorldState(dyn, x.keys, err)
    if isinstance(x, torch.Tensor):
        if not x.is_floating_point() or x.dim() == 0:
            return x
        m = _mask(pred, x.shape[env_dim]).to(x.device)
        shape = [1] * x.dim()
        shape[env_dim] = -1
        return torch.where(m.view(shape), torch.full_like(x, float("nan")), x)
    if isinstance(x, (tuple, list)):
        return type(x)(error_if(v, pred, env_dim) for v in x)
    if isinstance(x, dict):
        return {k: error_if(v, pred, env_dim) for k, v in x.items()}
    return x


def pre_condition(condition):
    """The inputs of envs failing `condition(*args, **kwargs)` (bool [B]) are
    NaN-guarded before the call (cotix/_design_by_contract.py:13-31)."""
    def decorator(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            bad = ~_as_mask(condition(*args, **kwargs))
            args = error_if(args, bad)
            kwargs = error_if(kwargs, bad)
            return func(*args, **kwargs)
        return wrapper
    return decorator


def post_condition(condition, provide_input=False):
    """The outputs of envs failing `condition(retval[, *args, **kwargs])` are
    NaN-guarded (cotix/_design_by_contract.py:34-57)."""
    def decorator(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            retval = func(*args, **kwargs)
            ok = condition(retval, *args, **kwargs) if provide_input else condition(retval)
            return error_if(retval, ~_as_mask(ok))
        return wrapper
    return decorator


def _as_mask(c):
    return torch.as_tensor(c).to(torch.bool) if not isinstance(c, bool) else torch.tensor(c)


def _check_all_annotations(obj):
    """Every annotated attribute has its annotated type (:60-68); a mismatch
    is a Python-level (trace-time) error, as in the reference."""
    for name, typ in getattr(type(obj), "__annotations__", {}).items():
        if isinstance(typ, type) and not isinstance(getattr(obj, name), typ):
            raise TypeError("%s=%r is not of type %s" % (name, getattr(obj, name), typ))


def class_invariant(cls):
    """Every public method first checks the annotations and then
    `self.__invariant__()` (cotix/_design_by_contract.py:80-107).  As in the
    reference, the error fires where __invariant__() is TRUE (its result is
    passed to eqx.error_if as the error condition); a per-env bool [B] NaN-
    guards only those envs of the attributes that are batched tensors /
    WorldStates (EQX_ON_ERROR=nan)."""
    def wrap(fn):
        @functools.wraps(fn)
        def wrapper(self, *args, **kwargs):
            _check_all_annotations(self)
            bad = self.__invariant__()
            if (isinstance(bad, bool) and bad) or (isinstance(bad, torch.Tensor) and bool(bad.any())):
                for name, val in list(vars(self).items()):
                    setattr(self, name, error_if(val, bad))
            return fn(self, *args, **kwargs)
        return wrapper
    for name in dir(cls):
        if name.startswith("_"):
            continue
        attr = getattr(cls, name)
        if callable(attr):
            setattr(cls, name, wrap(attr))
    return cls


ERR_STATE_NONFINITE = _ffi.ERR_STATE_NONFINITE
