"""ctypes binding of libcotix_amd.so (include/cotix_amd.h).

The product path has no fallback: if the HIP library is missing this module
raises ImportError, and every op raises RuntimeError on a non-zero return.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("COTIX_AMD_LIB", os.path.join(_HERE, "_lib", "libcotix_amd.so"))

# enums mirrored from include/cotix_amd.h
CIRCLE, AABB, POLYGON, POLYGON3, POLYGON4, POLYGON5, POLYGON6 = range(7)
FN_AABB_AABB, FN_CIRCLE_CIRCLE, FN_CIRCLE_AABB, FN_POLY_POLY, FN_AABB_POLY, FN_CIRCLE_POLY = range(6)
STAGE_EULER, STAGE_GRAVITY, STAGE_COLLIDER, STAGE_LUNAR, STAGE_ADVANCE_KEY = 1, 2, 4, 8, 16
STAGE_BROADPHASE = 32  # polygon-pair broadphase, results unchanged (include/cotix_amd.h)
SCENE_PER_ENV_BODY_PARAMS = 1  # cotix_scene_create_ex2 flag (include/cotix_amd.h)
STAGES_ROBOCUP = STAGE_EULER | STAGE_COLLIDER | STAGE_ADVANCE_KEY
STAGES_LUNAR = STAGE_EULER | STAGE_GRAVITY | STAGE_COLLIDER | STAGE_LUNAR | STAGE_ADVANCE_KEY
ERR_CIRCLE_AABB_CCP = 1
ERR_AABB_INVALID = 2
ERR_STATE_NONFINITE = 4

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
JUDGE_REGIONS = 4
MAX_STATE_WORDS = 96


class CotixJudge(ctypes.Structure):
    """struct cotix_judge (include/cotix_amd.h)."""
    _fields_ = [("rate_w", _F * MAX_STATE_WORDS), ("end_w", _F * MAX_STATE_WORDS), ("n_regions", _I),
                ("region_body", _I * JUDGE_REGIONS), ("region_lo", (_F * 6) * JUDGE_REGIONS),
                ("region_hi", (_F * 6) * JUDGE_REGIONS), ("region_reward", _F * JUDGE_REGIONS),
                ("done_on_error", _I), ("n_rate_regions", _I), ("rate_region_body", _I * JUDGE_REGIONS),
                ("rate_region_lo", (_F * 6) * JUDGE_REGIONS), ("rate_region_hi", (_F * 6) * JUDGE_REGIONS),
                ("rate_region_w", (_F * MAX_STATE_WORDS) * JUDGE_REGIONS),
                ("rate_region_bias", _F * JUDGE_REGIONS)]


class CotixControl(ctypes.Structure):
    """struct cotix_control (include/cotix_amd.h)."""
    _fields_ = [("body", _I), ("gain", (_F * 6) * 2), ("target", (_F * 6) * 2), ("bias", _F * 2),
                ("saturate", _I), ("clip_lo", _F * 2), ("clip_hi", _F * 2)]


SIGNATURES = {
    "cotix_params_default": (_I, [_P]),
    "cotix_scene_create": (_I, [_I, _P, _I, _P, _P, _P, ctypes.POINTER(_P)]),
    "cotix_scene_create_ex": (_I, [_I, _P, _I, _P, _P, _P, _P, ctypes.POINTER(_P)]),
    "cotix_scene_params": (_I, [_P, _P]),
    "cotix_scene_destroy": (_I, [_P]),
    "cotix_scene_geom_floats": (_I, [_P]),
    "cotix_scene_info": (_I, [_P, _P, _P, _P, _P]),
    "cotix_scene_set_variant": (_I, [_P, _I, _I]),
    "cotix_scene_variant": (_I, [_P, _P, _P]),
    "cotix_step": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P]),
    "cotix_step_autoreset": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _P, _P]),
    "cotix_step_ex": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P, _P, _P, _P, _P]),
    "cotix_eval": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, ctypes.POINTER(CotixJudge),
                        ctypes.POINTER(CotixControl), _P, _I, _P, _P, _I, _P, _P, _P, _P]),
    "cotix_rollout": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P, _P, _P, _P, _P]),
    "cotix_rollout_backward": (_I, [_P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P, _P, _P, _P]),
    "cotix_rollout_tape_words": (_I, [_P]),
    "cotix_rollout_ex": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P, _P, _P, _P, _P, _P]),
    "cotix_rollout_backward_ex": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _P, _I, _P, _P, _P, _P]),
    "cotix_body_penetration": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "cotix_body_aabb": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "cotix_physics_euler": (_I, [_P, _I, _I, _F, _P]),
    "cotix_collider_resolve": (_I, [_P, _P, _P, _P, _P, _I, _I, _P]),
    "cotix_lunar_constraints": (_I, [_P, _I, _P]),
    "cotix_contacts": (_I, [_I, _I, _P, _P, _P, _P, _P]),
    "cotix_contacts_ex": (_I, [_I, _I, _P, _P, _P, _P, _P, _P]),
    "cotix_resolve": (_I, [_I, _P, _P, _P, _P, _P, _P]),
    "cotix_resolve_ex": (_I, [_I, _P, _P, _P, _P, _P, _P, _P]),
    "cotix_gjk": (_I, [_I, _P, _P, _P, _P, _P, _P]),
    "cotix_gjk_ex": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cotix_scene_create_ex2": (_I, [_I, _P, _I, _P, _P, _P, _P, _I, ctypes.POINTER(_P)]),
    "cotix_scene_waves_per_group": (_I, [_P]),
    "cotix_epa": (_I, [_I, _P, _P, _P, _I, _P, _P]),
    "cotix_threefry2x32": (_I, [_P, _P, _P, _I, _P]),
    "cotix_random_split": (_I, [_P, _I, _I, _P, _P]),
    "cotix_random_split_ex": (_I, [_P, _I, _I, _I, _P, _P]),
    "cotix_random_uniform": (_I, [_P, _I, _I, _F, _F, _P, _P]),
    "cotix_random_uniform_ex": (_I, [_P, _I, _I, _F, _F, _I, _P, _P]),
    "cotix_order_clockwise": (_I, [_P, _I, _I, _P]),
    "cotix_observe": (_I, [_P, _I, _I, _P, _P]),
    "cotix_render_count": (_I, [_P]),
    "cotix_render": (_I, [_P, _P, _P, _I, _I, _P, _P]),
    "cotix_check_state": (_I, [_P, _I, _I, _P, _P]),
    "cotix_last_error": (ctypes.c_char_p, []),
    "cotix_version": (ctypes.c_char_p, []),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libcotix_amd.so not found at %s -- build it with `python __graft_entry__.py` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc, what=""):
    if rc != 0:
        raise RuntimeError("%s failed: %s" % (what, lib.cotix_last_error().decode()))
    return rc


def ptr(t):
    """Device pointer of a contiguous torch tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
