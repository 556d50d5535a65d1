"""Workload counters of the fused step (perf tooling): per wave-step active
phase-C items, candidate-scan rounds, resolutions and phase-F items, from the
host emulation of the kernel built with -DCOTIX_STATS.

  python tools/collider_stats.py [--scenario robocup|lunar] [--envs 256] [--steps 64] [--ew 4] [--broadphase]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "emu"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
LIB = "/tmp/libcotix_emu_stats.so"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="robocup")
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--ew", type=int, default=4)
    ap.add_argument("--broadphase", action="store_true", help="COTIX_STAGE_BROADPHASE (polygon scenes)")
    ap.add_argument("--drop", type=float, default=0.0, help="lunar: lower the lander and legs by this much (contact)")
    ap.add_argument("--settle", type=int, default=0, help="driver steps run first on the C port (lunar settles by ~2560)")
    a = ap.parse_args()
    src = os.path.join(ROOT, "tests", "emu", "cotix_emu.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
                    "-DCOTIX_STATS", "-w", src, "-o", LIB], check=True)
    import emu
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    lib = ctypes.CDLL(LIB)
    real = emu.load()  # the plain build: borrow its ctypes signatures
    for name in ("emu_scene_create", "emu_scene_create_ex", "emu_step"):
        getattr(lib, name).argtypes = getattr(real, name).argtypes
    lib.emu_last_error.restype = ctypes.c_char_p
    B = a.envs
    if a.scenario == "robocup":
        tr = np.load(os.path.join(ROOT, "tests", "golden", "robocup_trace.npz"))
        bodies = P.robocup_bodies()
        h, geom = emu.oracle_scene(lib, bodies)
        d0 = tr["dyn"][0]  # [8 envs][5][6]
        dyn = np.ascontiguousarray(np.concatenate([d0] * (B // d0.shape[0] + 1))[:B].transpose(1, 2, 0))
        stages, gstride = 1 | 4 | 16, 0
    else:
        tk = prng.split(prng.PRNGKey(0), B)
        rows, dyns = [], []
        for e in range(B):
            bodies = P.lunar_lander_bodies(tk[e])
            h, g = emu.oracle_scene(lib, bodies)
            rows.append(g)
            d = [b.dyn() for b in bodies]
            for b in range(3):
                d[b][1] -= a.drop
            dyns.append(d)
        geom = np.ascontiguousarray(np.stack(rows).astype(np.float32))
        gstride = geom.shape[1]
        dyn = np.ascontiguousarray(np.array(dyns, np.float32).transpose(1, 2, 0))
        stages = 1 | 2 | 4 | 8 | 16 | (32 if a.broadphase else 0)
    keys = np.ascontiguousarray(np.array(prng.split(prng.PRNGKey(3), B), np.uint32))
    dyn_reset = dyn.copy()
    err = np.zeros(B, np.uint32)
    if a.settle:  # the settled regime: advance on the C port (same bits), count the next steps only
        from cotix_oracle import cport
        src_bodies = P.robocup_bodies() if a.scenario == "robocup" else P.lunar_lander_bodies(prng.split(prng.PRNGKey(0), B)[0])
        sc = cport.Scene(cport.load(), src_bodies)
        sc.step(dyn, keys, err, a.settle, stages, geom=None if gstride == 0 else geom, dyn_reset=dyn_reset, nthreads=8)
    out = (ctypes.c_ulonglong * 17)()
    lib.emu_stats(out)
    emu.step(lib, h, dyn, keys, err, geom, gstride, a.steps, stages, E=a.ew, dyn_reset=dyn_reset)
    lib.emu_stats(out)
    ws = max(out[0], 1)
    print({"scenario": a.scenario, "envs": B, "steps": a.steps, "ew": a.ew,
           "active_items_per_wave_step": out[1] / ws, "rounds_per_wave_step": out[2] / ws,
           "resolutions_per_env_step": out[3] / (B * a.steps), "f_items_per_wave_step": out[4] / ws,
           "b_items_per_wave_step": out[5] / ws, "valid_draw_frac": out[7] / max(out[6], 1),
           "items_left_after_round1_per_wave_step": out[8] / ws,
           "resolution_levels_per_env_step": out[9] / (B * a.steps), "resolution_levels_per_wave_step": out[10] / ws,
           "sequential_slots_per_wave_step": out[11] / ws,
           "valid_candidates_of_active_items_per_wave_step": out[12] / ws, "fit64_frac": out[13] / ws,
           "bp_candidates_per_wave_step": out[14] / ws, "bp_guard_fail_frac": out[15] / max(out[14], 1),
           "epa_runs_per_wave_step": out[16] / ws})


if __name__ == "__main__":
    main()
