"""TEST INFRASTRUCTURE ONLY -- CPU oracle, never imported by the product path.

Restatement of the third-party ``jax.random`` primitives the cotix hot path
calls (jax/jaxlib >= 0.4.18, unpinned by the reference: ``pyproject.toml:16``).
Layouts: JAX's *legacy* (``jax_threefry_partitionable=False``) threefry
layout, the default of the 0.4.x line the reference pins as its floor, and
the *partitionable* one (the default from JAX 0.5), selected by the parameter
block in force (params.current().prng_layout):
  legacy         split(k, n) = threefry(k, iota(2n)) halves, reshaped (n, 2);
                 random_bits(k, (m,)) from the halves of iota(m) (zero pad if odd)
  partitionable  split(k, n)[i] = threefry(k, (0, i))  (_threefry_split_foldlike,
                 iota_2x32_shape's (hi, lo) counter words); random_bits word i
                 = y0 ^ y1 of threefry(k, (0, i))  (_threefry_random_bits_partitionable)

Call sites in the reference:
  split            cotix/_colliders.py:142,175,254,264,295 ; examples/test_viz.py:39
  bernoulli        cotix/_colliders.py:223-224
  choice(p=...)    cotix/_colliders.py:284
  normal           cotix/_geometry_utils.py:45 (via cotix/_collisions.py:288)
  uniform          cotix/_lunar_lander.py:110-123

Parity is pinned by external known-answer tests (Random123 threefry2x32-20
vectors and the published ``split(PRNGKey(0))`` value), see
tests/test_oracle_prng.py.  Everything else about jax.random here is a
restatement of its published algorithm (jax/_src/prng.py, jax/_src/random.py).
"""
import numpy as np

from . import params as _params

U32 = np.uint32
_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


def _rotl(v, r):
    return (v << U32(r)) | (v >> U32(32 - r))


def threefry2x32(key, x0, x1):
    """threefry2x32-20 block function, vectorised over counters.

    key: (k0, k1) uint32 scalars; x0, x1: uint32 arrays.  Returns (y0, y1).
    Restates jax/_src/prng.py ``_threefry2x32_lowering`` (5 x 4 rounds,
    key schedule ks = [k0, k1, k0^k1^0x1BD11BDA]).
    """
    with np.errstate(over="ignore"):
        k0 = U32(key[0])
        k1 = U32(key[1])
        ks = (k0, k1, U32(k0 ^ k1 ^ U32(0x1BD11BDA)))
        v0 = np.asarray(x0, dtype=U32) + ks[0]
        v1 = np.asarray(x1, dtype=U32) + ks[1]
        for g in range(5):
            for r in _ROT[g % 2]:
                v0 = v0 + v1
                v1 = _rotl(v1, r)
                v1 = v0 ^ v1
            v0 = v0 + ks[(g + 1) % 3]
            v1 = v1 + ks[(g + 2) % 3] + U32(g + 1)
        return v0.astype(U32), v1.astype(U32)


def PRNGKey(seed):
    """jax.random.PRNGKey(int) legacy seeding: (seed >> 32, seed & 0xffffffff)."""
    seed = int(seed)
    return np.array([(seed >> 32) & 0xFFFFFFFF if seed >= 0 else 0xFFFFFFFF,
                     seed & 0xFFFFFFFF], dtype=U32)


def _threefry_2x32_counts(key, counts):
    """jax/_src/prng.py ``threefry_2x32(keypair, count)``: split counts in two
    halves (zero pad when odd), run the block, concatenate, drop the pad."""
    counts = np.asarray(counts, dtype=U32).ravel()
    odd = counts.size % 2
    if odd:
        counts = np.concatenate([counts, np.zeros(1, U32)])
    h = counts.size // 2
    y0, y1 = threefry2x32(key, counts[:h], counts[h:])
    out = np.concatenate([y0, y1])
    return out[:-1] if odd else out


def _partitionable():
    return _params.current().partitionable


def split(key, num=2):
    """jax.random.split(key, num): legacy layout iota(2n) counters;
    partitionable: key i = threefry(key, (0, i))."""
    if _partitionable():
        y0, y1 = threefry2x32(key, np.zeros(num, U32), np.arange(num, dtype=U32))
        return np.stack([y0, y1], 1).astype(U32)
    out = _threefry_2x32_counts(key, np.arange(2 * num, dtype=U32))
    return out.reshape(num, 2)


def split_at(key, num, idx):
    """Element ``idx`` of ``split(key, num)`` computed with two blocks only
    (what the device code does).  Key k = (flat[2k], flat[2k+1]) where flat
    = y0 || y1 of blocks b < num with counter (b, num + b); partitionable:
    the one block (0, idx)."""
    if _partitionable():
        y0, y1 = threefry2x32(key, np.array([0], U32), np.array([idx], U32))
        return np.array([y0[0], y1[0]], dtype=U32)
    words = []
    for m in (2 * idx, 2 * idx + 1):
        if m < num:
            y0, _ = threefry2x32(key, np.array([m], U32), np.array([num + m], U32))
            words.append(y0[0])
        else:
            b = m - num
            _, y1 = threefry2x32(key, np.array([b], U32), np.array([num + b], U32))
            words.append(y1[0])
    return np.array(words, dtype=U32)


def random_bits(key, shape):
    """``jax.random.bits`` / ``_random_bits`` for 32-bit words, in the layout
    in force."""
    size = int(np.prod(shape)) if len(shape) else 1
    if _partitionable():
        y0, y1 = threefry2x32(key, np.zeros(size, U32), np.arange(size, dtype=U32))
        return (y0 ^ y1).astype(U32).reshape(shape)
    return _threefry_2x32_counts(key, np.arange(size, dtype=U32)).reshape(shape)


def bits_to_unit_float(bits):
    """(bits >> 9) | 0x3F800000 reinterpreted as f32, minus 1 -> [0, 1)."""
    fb = (np.asarray(bits, dtype=U32) >> U32(9)) | U32(0x3F800000)
    return fb.view(np.float32) - np.float32(1.0)


def uniform(key, shape=(), minval=0.0, maxval=1.0):
    """jax.random.uniform (f32): floats * (maxval - minval) + minval, then
    lax.max(minval, .)."""
    lo = np.float32(minval)
    hi = np.float32(maxval)
    f = bits_to_unit_float(random_bits(key, shape))
    with np.errstate(all="ignore"):
        v = f * (hi - lo) + lo
    return np.maximum(lo, v).astype(np.float32).reshape(shape)


def bernoulli_half(key):
    """jax.random.bernoulli(key, 0.5, ()) == uniform(key) < 0.5
    <=> the top bit of the single random word is 0."""
    return bool(uniform(key, ()) < np.float32(0.5))


def bernoulli(key, p):
    """jax.random.bernoulli(key, p, ()) == uniform(key) < p (p as f32)."""
    return bool(uniform(key, ()) < np.float32(p))


def cumsum_assoc(x):
    """jnp.cumsum on CPU lowers through lax.associative_scan (the
    reduce-window form is TPU-only): restate its pairwise order exactly."""
    x = [np.float32(v) for v in x]

    def scan(e):
        n = len(e)
        if n < 2:
            return list(e)
        reduced = [e[2 * k] + e[2 * k + 1] for k in range(n // 2)]
        odd = scan(reduced)
        if n % 2 == 0:
            even = [odd[k] + e[2 * k + 2] for k in range(len(odd) - 1)]
        else:
            even = [odd[k] + e[2 * k + 2] for k in range(len(odd))]
        even = [e[0]] + even
        out = []
        for k in range(n):
            out.append(even[k // 2] if k % 2 == 0 else odd[k // 2])
        return out

    return [np.float32(v) for v in scan(x)]


def choice_p(key, n, p):
    """jax.random.choice(key, arange(n), p=p) with replace=True, shape=():
    r = cumsum(p)[-1] * (1 - uniform(key)); index = searchsorted(cumsum, r,
    side='left')."""
    c = cumsum_assoc(p)
    u = uniform(key, ())
    r = np.float32(c[-1] * (np.float32(1.0) - np.float32(u)))
    for k in range(n):
        if not (c[k] < r):  # first k with r <= c[k]; NaN compares false -> k
            return k
    return n


_ERFINV_LT5 = (2.81022636e-08, 3.43273939e-07, -3.5233877e-06, -4.39150654e-06,
               0.00021858087, -0.00125372503, -0.00417768164, 0.246640727, 1.50140941)
_ERFINV_GE5 = (-0.000200214257, 0.000100950558, 0.00134934322, -0.00367342844,
               0.00573950773, -0.0076224613, 0.00943887047, 1.00167406, 2.83297682)


def erf_inv32(x):
    """XLA's f32 ErfInv (Giles polynomial, xla/client/lib/math.cc ErfInv32):
    w = -log1p(-x*x); w<5: poly(w-2.5) else poly(sqrt(w)-3); result p*x."""
    f = np.float32
    x = f(x)
    with np.errstate(all="ignore"):
        w = -np.log1p(-x * x)
        lt = bool(w < f(5.0))
        c = _ERFINV_LT5 if lt else _ERFINV_GE5
        w = (w - f(2.5)) if lt else (np.sqrt(w) - f(3.0))
        p = f(c[0])
        for i in range(1, 9):
            p = f(c[i]) + p * w
        return f(p * x)


def normal(key, shape):
    """jax.random.normal (f32): sqrt(2) * erf_inv(uniform(key, shape,
    nextafter(-1, 0), 1)).  Pinned: reproduces the 13 published values of
    normal(PRNGKey(0), (10,)) and normal(PRNGKey(0), (3,)) bit for bit."""
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    u = uniform(key, shape, lo, 1.0).ravel()
    out = np.array([np.float32(np.sqrt(2.0)) * erf_inv32(v) for v in u], dtype=np.float32)
    return out.reshape(shape)


def log1p_cr32(a):
    """log1p of an f32, correctly rounded to f32 (the f64 log1p rounded once).
    The device's random_direction uses the same (cx::log1p_cr); numpy's f32
    log1p is the host's vector math library (SVML under AVX-512), which no
    device code can reproduce bit for bit."""
    with np.errstate(all="ignore"):
        return np.float32(np.log1p(np.float64(np.float32(a))))


def erf_inv32_cr(x):
    """erf_inv32 with log1p_cr32 for its log1p (w = -log1p(-x*x)); the rest
    is XLA's f32 ErfInv as in erf_inv32.  Reproduces the same 13 published
    jax.random.normal values (tests/test_oracle_prng.py)."""
    f = np.float32
    x = f(x)
    with np.errstate(all="ignore"):
        w = -log1p_cr32(-x * x)
        lt = bool(w < f(5.0))
        c = _ERFINV_LT5 if lt else _ERFINV_GE5
        w = (w - f(2.5)) if lt else (np.sqrt(w) - f(3.0))
        p = f(c[0])
        for i in range(1, 9):
            p = f(c[i]) + p * w
        return f(p * x)


def random_direction(key):
    """random_direction(key) (cotix/_geometry_utils.py:37-46) for any key:
    x / ||x|| with x = normal(key, (2,)) through erf_inv32_cr, in the PRNG
    layout in force.  PRNGKey(1) -- the key check_for_collision_convex uses
    when given none (cotix/_collisions.py:287-288) -- is the constant
    gjk_initial_direction(), so that key=None and key=PRNGKey(1) agree as in
    the reference (the two log1p forms differ there by 2 ulp in x; XLA's own
    log1p is not pinned by any published value)."""
    k = np.asarray(key, dtype=U32).reshape(2)
    if int(k[0]) == 0 and int(k[1]) == 1:
        return gjk_initial_direction()
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    u = uniform(k, (2,), lo, 1.0)
    x = [np.float32(np.float32(np.sqrt(2.0)) * erf_inv32_cr(v)) for v in u]
    with np.errstate(all="ignore"):
        n = np.sqrt(np.float32(x[0] * x[0] + x[1] * x[1]))
        return (np.float32(x[0] / n), np.float32(x[1] / n))


def gjk_start_direction(initial_direction=None, key=None):
    """check_for_collision_convex's start direction (cotix/_collisions.py:
    285-298): rnd = random_direction(key or PRNGKey(1)); rnd if
    initial_direction has a NaN (its default) else rnd * 0.1 +
    initial_direction * 0.9, in f32."""
    rnd = gjk_initial_direction() if key is None else random_direction(key)
    if initial_direction is None:
        return rnd
    d = [np.float32(v) for v in initial_direction]
    if np.isnan(d[0]) or np.isnan(d[1]):
        return rnd
    with np.errstate(all="ignore"):
        return tuple(np.float32(np.float32(r * np.float32(0.1)) + np.float32(v * np.float32(0.9)))
                     for r, v in zip(rnd, d))


def gjk_initial_direction():
    """random_direction(PRNGKey(1)) (cotix/_geometry_utils.py:37-46 called from
    cotix/_collisions.py:287-298): x / ||x|| with x = normal(PRNGKey(1), (2,)).
    Constant for every GJK call: legacy layout (-0.05243401, 0.9986244) =
    (0xbd56c50b, 0x3f7fa5d9); partitionable (-0.8767744, 0.4809021) =
    (0xbf607449, 0x3ef638cd)."""
    x = normal(PRNGKey(1), (2,))
    n = np.sqrt(x[0] * x[0] + x[1] * x[1])
    return (np.float32(x[0] / n), np.float32(x[1] / n))
