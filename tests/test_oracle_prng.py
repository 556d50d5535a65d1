"""Pins the oracle's jax.random restatement (oracle/cotix_oracle/prng.py)
against external known-answer vectors -- no reference test pins the PRNG
(SURVEY.md 8c), so these are the anchors."""
import numpy as np

from cotix_oracle import prng

U = np.uint32


def _blk(k, c):
    y0, y1 = prng.threefry2x32(k, np.array([c[0]], U), np.array([c[1]], U))
    return int(y0[0]), int(y1[0])


def test_threefry_random123_kat():
    assert _blk((0, 0), (0, 0)) == (0x6B200159, 0x99BA4EFE)
    assert _blk((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF)) == (0x1CB996FC, 0xBB002BE7)
    assert _blk((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3)) == (0xC4923A9C, 0x483DF7A0)


def test_split_published_value():
    assert prng.split(prng.PRNGKey(0)).tolist() == [[4146024105, 967050713], [2718843009, 1272950319]]


def test_split_at_matches_split():
    for seed in (0, 1, 7):
        k = prng.PRNGKey(seed)
        for n in (1, 2, 3, 5, 8, 22):
            s = prng.split(k, n)
            for i in range(n):
                assert (prng.split_at(k, n, i) == s[i]).all()


def test_uniform_published_value():
    # jax.random.uniform(PRNGKey(0), (3,)) from the JAX documentation
    u = prng.uniform(prng.PRNGKey(0), (3,))
    assert u.tolist() == np.array([0.9653214, 0.31468165, 0.63302994], np.float32).tolist()


def test_normal_published_values():
    # jax.random.normal(PRNGKey(0), (10,)) / (3,) from the JAX documentation
    n10 = prng.normal(prng.PRNGKey(0), (10,))
    exp10 = np.array([-0.3721109, 0.26423115, -0.18252768, -0.7368197, -0.44030377,
                      -0.1521442, -0.67135346, -0.5908641, 0.73168886, 0.5673026], np.float32)
    assert n10.tolist() == exp10.tolist()
    n3 = prng.normal(prng.PRNGKey(0), (3,))
    assert n3.tolist() == np.array([1.8160863, -0.48262316, 0.33988908], np.float32).tolist()


def test_gjk_initial_direction_constant():
    d = prng.gjk_initial_direction()
    assert [int(np.float32(v).view(U)) for v in d] == [0xBD56C50B, 0x3F7FA5D9]


def test_bernoulli_is_top_bit():
    k = prng.PRNGKey(5)
    for key in prng.split(k, 64):
        bits = prng.random_bits(key, ())
        assert prng.bernoulli_half(key) == (int(bits) >> 31 == 0)


def test_choice_never_picks_zero_probability():
    keys = prng.split(prng.PRNGKey(11), 200)
    p = [np.float32(0.0), np.float32(1 / 3), np.float32(0.0), np.float32(1 / 3), np.float32(1 / 3)]
    for key in keys:
        assert prng.choice_p(key, 5, p) in (1, 3, 4)


def test_cumsum_associative_order():
    x = [np.float32(v) for v in (0.1, 0.2, 0.3, 0.4, 0.5)]
    c = prng.cumsum_assoc(x)
    f = np.float32
    assert c[3] == (x[0] + x[1]) + (x[2] + x[3])
    assert c[4] == ((x[0] + x[1]) + (x[2] + x[3])) + x[4]
    assert c[2] == (x[0] + x[1]) + x[2]
    assert c[0] == x[0] and isinstance(c[0], f)
