"""Per-phase cycle profile of the fused step kernel (perf tooling, not the
product).  Needs the profiling build of the library:
    hipcc ... -DCOTIX_PHASE_PROF -> parallax_amd/_lib/libcotix_amd_prof.so   (tools/phase_prof.py --build)
and runs the bench workload with it:  python tools/phase_prof.py [--scenario robocup|lunar|box] [--launches N]
--mode grad: the config-5 rollout (cotix_rollout forward + cotix_rollout_backward,
--substeps steps), the forward's and the backward's phases reported apart."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "parallax_amd", "_lib", "libcotix_amd_prof.so")
NAMES = ["load", "save", "A", "T", "B", "C0", "C0b", "C1", "C2", "C3", "D", "E", "ret", "store", "restore", "G",
         "adj", "F", "K", "E1", "R", "trace", "B0", "B1", "F0", "F1", "F2", "F3",
         "TV0", "TV1", "TV2", "TV3", "J", "GE", "sub0", "sub1", "sub2", "sub3", "sub4", "sub5", "sub6", "sub7"]


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    g.build_hip(out=LIB, defines=("COTIX_PHASE_PROF", "COTIX_EW4_ONLY"), ews=(4,))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--scenario", default="robocup")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--substeps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=1, help="untimed launches first (lunar settles after ~40)")
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--no-broadphase", action="store_true", help="lunar: without COTIX_STAGE_BROADPHASE")
    ap.add_argument("--drop", type=float, default=0.0, help="lunar: lower lander and legs by this much (in contact)")
    ap.add_argument("--mode", default="step", choices=["step", "grad"])
    ap.add_argument("--fwd-skip", type=int, default=0,
                    help="grad: COTIX_DEBUG_SKIP bits for the forward only (tooling build; timing experiments)")
    a = ap.parse_args()
    if a.build:
        return build()
    os.environ["COTIX_AMD_LIB"] = os.path.abspath(a.lib)
    # the one-wave kernels only: the phase-profiling build of step_help_kernel
    # (build 0ac7b676) constructs its WaveRun without the cycle accumulators,
    # so its phases write through a null pointer (a GPU memory fault on the
    # r06z box); the per-phase cycles are the step wave's program either way
    os.environ["COTIX_KEY_HELPER"] = "0"
    os.environ["COTIX_SPLIT_BWD"] = "0"
    sys.path.insert(0, ROOT)
    import torch
    import parallax_amd as pa
    f = pa._ffi.lib.cotix_phase_cycles
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    B = a.envs
    if a.scenario == "robocup":
        keys = pa.random.split(pa.random.PRNGKey(3, dev), B).contiguous()
        scen = pa.RoboCupEnv(batch=B, device=dev, keys=keys, perturb=True)
    elif a.scenario == "box":
        scen = pa.BoxWorld(batch=B, device=dev)
    else:
        tk = pa.random.split(pa.random.PRNGKey(0, dev), B).contiguous()
        ck = pa.random.split(pa.random.PRNGKey(1, dev), B).contiguous()
        scen = pa.LunarLander(key=tk, batch=B, device=dev, collider_keys=ck)
        if a.no_broadphase:
            scen.stages &= ~pa._ffi.STAGE_BROADPHASE
        if a.drop:
            for i in range(3):
                scen.dyn_reset[i, 1] -= a.drop
                scen.dyn_reset[i, 3] = -0.3
    ew = 4  # the profiling build carries the default tiling only (COTIX_EW4_ONLY)
    waves = (B + ew - 1) // ew
    buf = (ctypes.c_ulonglong * 48)()

    def phases(steps):
        n = f(buf, 48)
        nph = NAMES.index("sub0")
        tot = sum(buf[q] for q in range(min(n, nph)))  # the sub-phase timers (nph..) overlap the phases
        return {"cycles_per_wave_step_total": tot / waves / steps,
                "phases": {NAMES[q]: {"cycles_per_wave_step": buf[q] / waves / steps, "share": buf[q] / tot}
                           for q in range(n) if buf[q]}}

    if a.mode == "grad":
        world = scen.world
        nb = len(world.bodies)
        stages, ab = pa._ffi.STAGES_ROBOCUP, nb - 1
        if a.scenario == "lunar":  # bench.py grad_lunar: settled on the terrain, the lander's dv and x
            stages, ab = scen.stages, 0
            for _ in range(40):
                world.step(64, 1e-2, stages)
        dyn0, keys0 = world.dyn.clone(), world.keys.clone()
        gen = torch.Generator(device="cpu").manual_seed(1234)
        actions = (torch.randn(a.substeps, B, 2, generator=gen) * 0.1).to(dev)
        w = pa.rollout.ball_x_weights(nb, ab)
        fwd, bwd = [], []
        for it in range(a.warmup + a.launches):
            world.dyn.copy_(dyn0)
            world.keys.copy_(keys0)
            world.err.zero_()
            torch.cuda.synchronize()
            f(buf, 48)
            os.environ["COTIX_DEBUG_SKIP"] = str(a.fwd_skip)
            _, saved = pa.rollout_forward(world, actions, ab, w, stages=stages)
            torch.cuda.synchronize()
            os.environ["COTIX_DEBUG_SKIP"] = "0"
            pf = phases(a.substeps)
            if a.fwd_skip == 0:  # (a skipped save leaves the saved state / tape unwritten: no backward)
                pa.rollout_backward(world, saved)
                torch.cuda.synchronize()
            pb = phases(a.substeps)
            if it >= a.warmup:
                fwd.append(pf)
                bwd.append(pb)
        print(json.dumps({"scenario": a.scenario, "mode": "grad", "envs": B, "envs_per_wave": ew,
                          "steps_per_launch": a.substeps, "forward": fwd[-1], "backward": bwd[-1]}, indent=1))
        return
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    for _ in range(a.warmup):
        env.step(a.substeps)
    f(buf, 48)  # reset after warm-up
    for _ in range(a.launches):
        env.step(a.substeps)
    torch.cuda.synchronize()
    p = phases(a.launches * a.substeps)
    print(json.dumps({"scenario": a.scenario, "envs": B, "envs_per_wave": ew, **p}, indent=1))


if __name__ == "__main__":
    main()
