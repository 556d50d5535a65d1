"""jax.random surface used by cotix, executed by the HIP PRNG kernels.

Keys are int32 tensors [..., 2] holding the uint32 bit patterns of JAX's
threefry keys (uint32 arithmetic happens only in the kernels).  ``layout``:
"legacy" (jax_threefry_partitionable=False, the default here and in JAX
0.4.x), "partitionable" (the default from JAX 0.5), or a Params (its
prng_layout) -- include/cotix_amd.h COTIX_PRNG_*.
Call sites replaced: cotix/_colliders.py:142-295, cotix/_lunar_lander.py:109-123,
examples/test_viz.py:39,46.
"""
import torch

from . import _ffi
from .params import layout_id


def PRNGKey(seed, device="cuda"):
    """jax.random.PRNGKey(int) (legacy): (seed >> 32, seed & 0xffffffff)."""
    seed = int(seed)
    hi = (seed >> 32) & 0xFFFFFFFF if seed >= 0 else 0xFFFFFFFF
    lo = seed & 0xFFFFFFFF
    to_i32 = lambda u: u - (1 << 32) if u >= (1 << 31) else u  # noqa: E731
    return torch.tensor([to_i32(hi), to_i32(lo)], dtype=torch.int32, device=device)


def _keys2d(keys):
    if keys.dtype != torch.int32 or keys.shape[-1] != 2:
        raise ValueError("keys must be int32 [..., 2]")
    return keys.reshape(-1, 2).contiguous()


def split(keys, num=2, layout=None):
    """jax.random.split(key, num) for every key of a [..., 2] batch."""
    k = _keys2d(keys)
    out = torch.empty((k.shape[0], num, 2), dtype=torch.int32, device=k.device)
    _ffi.check(_ffi.lib.cotix_random_split_ex(_ffi.ptr(k), k.shape[0], num, layout_id(layout), _ffi.ptr(out),
                                              _ffi.stream_ptr(k.device)), "cotix_random_split_ex")
    return out.reshape(*keys.shape[:-1], num, 2)


def uniform(keys, count=None, minval=0.0, maxval=1.0, layout=None):
    """jax.random.uniform(key, (count,) or (), minval, maxval) (f32) per key."""
    k = _keys2d(keys)
    n = 1 if count is None else int(count)
    out = torch.empty((k.shape[0], n), dtype=torch.float32, device=k.device)
    _ffi.check(_ffi.lib.cotix_random_uniform_ex(_ffi.ptr(k), k.shape[0], n, float(minval), float(maxval),
                                                layout_id(layout), _ffi.ptr(out), _ffi.stream_ptr(k.device)),
               "cotix_random_uniform_ex")
    shape = keys.shape[:-1] if count is None else (*keys.shape[:-1], n)
    return out.reshape(shape)


def threefry2x32(keys, counters):
    """Raw threefry2x32-20 blocks: keys, counters int32 [n, 2] -> [n, 2]."""
    k = _keys2d(keys)
    c = counters.reshape(-1, 2).contiguous()
    out = torch.empty_like(k)
    _ffi.check(_ffi.lib.cotix_threefry2x32(_ffi.ptr(k), _ffi.ptr(c), _ffi.ptr(out), k.shape[0],
                                           _ffi.stream_ptr(k.device)), "cotix_threefry2x32")
    return out
