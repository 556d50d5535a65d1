"""Parameter blocks (include/cotix_amd.h cotix_params) the parity tests run
the path under: the reference's literals (""), the partitionable PRNG layout
("_part", the default of JAX >= 0.5), and a non-default constant set ("_alt":
Baumgarte 0.2 / 0.02, bernoulli p 0.3, GJK capped at 1 step, EPA at 3
iterations).  The suffix names the golden fixtures made under each
(tests/golden/make_golden.py)."""
PARAM_SETS = {
    "": {},
    "_part": {"prng_layout": "partitionable"},
    "_alt": {"baumgarte": 0.2, "baumgarte_dt": 0.02, "contact_p": 0.3, "gjk_max_steps": 1, "epa_max_iters": 3},
}


def oracle_params(suffix):
    from cotix_oracle import params
    return params.Params(**PARAM_SETS[suffix])


def host_params(suffix):
    import parallax_amd as pa
    return pa.Params(**PARAM_SETS[suffix])
