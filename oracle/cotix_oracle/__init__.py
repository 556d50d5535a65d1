"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the cotix hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker.  The product path
(parallax_amd) never imports it.
"""
from . import geometry, physics, prng  # noqa: F401
