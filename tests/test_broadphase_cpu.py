"""The polygon broadphase (COTIX_STAGE_BROADPHASE) is exact: on the
adversarial sets of tests/bp_cases.py the step kernel's program (host
emulation) with the broadphase equals the C port of the oracle (no
broadphase) bit for bit -- state, keys, err and the collider trace, whose
cells show every contact's NaN-ness.  Mutation builds of the same kernel
source show what the test detects: margin 0 drops the reference's contacts
at positive gaps (the touch set) and fails; the margin halved and the shape
guard removed still pass, as DESIGN.md section 3 explains (the margin has
~2^8 headroom over the rounding bound; without the guard exactness rests on
GJK rejecting, which the argument does not need but which holds on every
case searched)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bp_cases as C

HERE = os.path.dirname(os.path.abspath(__file__))
EMU = os.path.join(HERE, "emu")
F = np.float32
STAGES = 1 | 4 | 16


def _build(name, defines):
    out = os.path.join(EMU, "build", name)
    src = os.path.join(EMU, "cotix_emu.cpp")
    hdr = [os.path.join(HERE, "..", "parallax_amd", "csrc", f) for f in ("cotix_kernel.h", "cotix_device.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(f) for f in [src] + hdr):
        tmp = "%s.%d.tmp" % (out, os.getpid())  # parallel workers: build privately, then rename atomically
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-w",
                        *["-D" + d for d in defines], src, "-o", tmp], check=True)
        os.replace(tmp, out)
    return out


@pytest.fixture(scope="module")
def libs():
    import ctypes
    subprocess.run(["make", "-s", "-C", EMU, "build/libcotix_emu.so"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "..", "oracle")], check=True)
    sys.path.insert(0, EMU)
    import emu
    real = emu.load()
    out = {"plain": real}
    for name, d in (("margin0", ["COTIX_BP_MARGIN_MUL=0.0f"]), ("margin_half", ["COTIX_BP_MARGIN_MUL=0.5f"]),
                    ("noguard", ["COTIX_BP_GUARD=0"]), ("stats", ["COTIX_STATS"])):
        lib = ctypes.CDLL(_build("libcotix_emu_bp_%s.so" % name, d))
        for fn in ("emu_scene_create", "emu_step", "emu_step_ex"):
            getattr(lib, fn).argtypes = getattr(real, fn).argtypes
        out[name] = lib
    return emu, out


def _sets():
    g = C.load_touch()
    yield "touch44", g["touch_44_a"], g["touch_44_b"]
    yield "touch46", g["touch_46_a"], g["touch_46_b"]
    for k, name in enumerate(("collinear", "sliver", "far", "nonfinite")):
        for na, nb in ((4, 4), (4, 6)):
            A, B = C.gen_set(name, na, nb, 48, 10 * k + nb)
            yield "%s%d%d" % (name, na, nb), A, B


SETS = {name: (A, B) for name, A, B in _sets()}


def run_emu(emu, lib, A, B, bp=True):
    bodies = C.scene_bodies(A.shape[1], B.shape[1])
    h, _ = emu.oracle_scene(lib, bodies)
    geom = C.geometry_rows(A, B)
    n = A.shape[0]
    dyn = np.zeros((2, 6, n), F)
    keys = np.ascontiguousarray(np.stack([np.arange(n), np.arange(n) * 7 + 1], 1).astype(np.uint32))
    err = np.zeros(n, np.uint32)
    ch, cl = emu.step_ex(lib, h, dyn, keys, err, geom, geom.shape[1], 1, STAGES | (32 if bp else 0), 2, E=4)
    return dyn, keys, err, ch, cl


def run_cport(A, B):
    from cotix_oracle import cport
    lib = cport.load()
    sc = cport.Scene(lib, C.scene_bodies(A.shape[1], B.shape[1]))
    geom = C.geometry_rows(A, B)
    n = A.shape[0]
    dyn = np.zeros((2, 6, n), F)
    keys = np.ascontiguousarray(np.stack([np.arange(n), np.arange(n) * 7 + 1], 1).astype(np.uint32))
    err = np.zeros(n, np.uint32)
    ch, cl = sc.step_ex(dyn, keys, err, 1, STAGES, geom=geom, trace=True, nthreads=1)
    return dyn, keys, err, ch, cl


def same(a, b):
    a, b = np.asarray(a, F), np.asarray(b, F)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def agree(x, y):
    return (same(x[0], y[0]) and np.array_equal(x[1], y[1]) and np.array_equal(x[2], y[2])
            and np.array_equal(x[3], y[3]) and np.array_equal(x[4], y[4]))


@pytest.mark.parametrize("name", sorted(SETS))
def test_broadphase_exact_on_adversarial_sets(libs, name):
    emu, L = libs
    A, B = SETS[name]
    want = run_cport(A, B)
    assert agree(run_emu(emu, L["plain"], A, B, bp=True), want), name
    assert agree(run_emu(emu, L["plain"], A, B, bp=False), want), name
    if name.startswith("touch"):  # the witnesses: contacts (cells) the reference HAS at a positive gap
        assert (want[4] >= 0).any()


def test_sets_exercise_the_broadphase(libs):
    """The separated sets reach the skip decision (stats build): pairs past
    the gap test, and most certified by the shape guard."""
    emu, L = libs
    import ctypes
    out = (ctypes.c_ulonglong * 32)()  # emu_stats writes (and returns) its counter count, 17 today
    L["stats"].emu_stats(out)
    for name in ("collinear44", "sliver46", "far46"):
        A, B = SETS[name]
        run_emu(emu, L["stats"], A, B)
    L["stats"].emu_stats(out)
    assert out[14] >= 3 * 48 * 0.5, list(out)
    assert out[15] < out[14], list(out)


def test_mutation_margin_zero_is_detected(libs):
    """A broadphase skipping every pair with a positive gap (margin 0) drops
    the touch witnesses' contacts: the comparison must fail."""
    emu, L = libs
    bad = 0
    for name in ("touch44", "touch46"):
        A, B = SETS[name]
        bad += not agree(run_emu(emu, L["margin0"], A, B), run_cport(A, B))
    assert bad > 0


def test_mutations_within_the_argument_pass(libs):
    """Margin halved / shape guard removed: still exact on every set (the
    margin's headroom, and GJK rejecting separated pairs) -- recorded so that
    a change in either shows up here."""
    emu, L = libs
    for lib in ("margin_half", "noguard"):
        for name in sorted(SETS):
            A, B = SETS[name]
            assert agree(run_emu(emu, L[lib], A, B), run_cport(A, B)), (lib, name)
