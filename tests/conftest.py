import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

_GPU_TESTS_RUN = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def d0():
    from cotix_oracle import prng
    return prng.gjk_initial_direction()


def pytest_runtest_setup(item):
    if item.get_closest_marker("gpu") is not None:
        _GPU_TESTS_RUN.append(item.nodeid)


def loaded_native_libraries():
    """Real paths of the shared objects mapped into this process."""
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and (parts[5].endswith(".so") or ".so." in parts[5]):
                out.add(os.path.realpath(parts[5]))
    return out


def pytest_sessionfinish(session, exitstatus):
    """Session-level check for -m gpu runs: the HIP library the product path
    binds (parallax_amd._ffi.LIB_PATH) must be the one mapped in this
    process -- a green GPU run that never loaded libcotix_amd.so (a silent
    fallback, a stale COTIX_AMD_LIB) fails here."""
    if not _GPU_TESTS_RUN:
        return
    from parallax_amd import _ffi
    want = os.path.realpath(_ffi.LIB_PATH)
    default = os.path.realpath(os.path.join(ROOT, "parallax_amd", "_lib", "libcotix_amd.so"))
    maps = loaded_native_libraries()
    problems = []
    if want not in maps:
        problems.append("%s is not mapped into the test process" % want)
    if want != default:
        problems.append("COTIX_AMD_LIB points away from the in-tree build (%s != %s)" % (want, default))
    tr = session.config.pluginmanager.get_plugin("terminalreporter")
    if problems:
        if tr is not None:
            tr.write_line("NATIVE LIBRARY CHECK FAILED: " + "; ".join(problems), red=True)
        session.exitstatus = 1
    elif tr is not None:
        tr.write_line("native library check: %s mapped (%s), %d gpu tests"
                      % (want, _ffi.lib.cotix_version().decode(), len(_GPU_TESTS_RUN)))


def pytest_terminal_summary(terminalreporter):
    """The gradient checks' measured errors (tests/grad_cases.py close): per
    workload, the floor its compared blocks needed at rtol 1e-5 -- the
    numbers DESIGN.md section 5 records against the tolerances."""
    gc = sys.modules.get("grad_cases")
    if gc is None or not getattr(gc, "MEASURED", None):
        return
    terminalreporter.write_line("gradient checks, floor needed at rtol 1e-5 (allowed: analytic %g, polygon %g):"
                                % (gc.ANALYTIC_TOL[1], gc.POLYGON_TOL[1]))
    for k in sorted(gc.MEASURED):
        terminalreporter.write_line("  %-22s %.3g" % (k, gc.MEASURED[k]))
