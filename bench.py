"""Benchmark: RoboCup, 4096 envs per GPU, env-steps/s (BASELINE.json metric).

One bench "step" = one launch of the fused HIP step kernel advancing every
env by --substeps driver steps (examples/test_viz.py:61-69: Euler ->
RandomizedCollider -> identity constraint pass -> key split), with episode
restarts on the reference's error_if trip (DESIGN.md "Measurement").  Inputs
are resident in HBM before the timed region.  value = envs * substeps * steps
* n_gpus / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W --substeps S --scenario robocup|lunar]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

Rank r owns the envs with global ids [r*B, (r+1)*B) of the N*B-env run and
builds them from those ids (RoboCupEnv(env_offset, total_envs)).  After each
launch the observation tensor is all-gathered over RCCL (asynchronous, double
buffered), the north star's one collective.

The JSON line also carries, measured in the same process after the headline
(rank 0, --extras auto):
  workload_stats  finite-env fraction and restarts per env-step of the headline
                  workload (the reference's RoboCup goes NaN at step 1)
  k1              the headline scene with ONE driver step per launch (the launch
                  rate an RL loop with per-step actions sees)
  finite_scene    BoxWorld (balls in a box, finite dynamics) at the same size
  lunar           BASELINE config 2 (LunarLander, 4096 envs, GJK/EPA) while the
                  landers fall; lunar_contact: settled on the terrain
  grad            BASELINE config 5 (64-step differentiable rollout, fwd + bwd);
                  grad_box: the same on the box world (finite gradients);
                  grad_lunar: LunarLander settled on its terrain (gradients
                  through GJK/EPA polygon contacts and the joints)
  eval            AbstractEnvironment.eval with a device judge and control,
                  4 NFEs x 16 env-steps in one cotix_eval launch
  config1         BASELINE config 1 (one LunarLander env, 10,000 steps): GPU
                  and the C port on one core
  roofline        primary bound = VALU issue (SQ_INSTS_VALU of the committed
                  rocprofv3 pass of this workload / live launch time), HBM
                  figures as the north star asks

--mode grad (BASELINE config 5) as its own line: one bench step = a
differentiable --substeps (64) step RoboCup rollout, forward (cotix_rollout)
+ backward (cotix_rollout_backward) -> d(sum_t ball x)/d(action) for every env.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
# the C port's OpenMP threads (CPU baseline) sleep when idle instead of
# spinning on the cores the GPU-launching thread runs on
os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD per
# 2 cycles (SIMD-32) at 2.4 GHz (MI355X_MICROARCH.md); one wave alone issues
# one per 4 cycles, so at one wave per SIMD the ceiling is half of this.
VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--substeps", type=int, default=64)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--scenario", default="robocup", choices=["robocup", "lunar", "box"])
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--extras", default="auto", choices=["auto", "off"])
    ap.add_argument("--mode", default="step", choices=["step", "grad"])
    ap.add_argument("--dump-gather", default=None, help="save the last all-gathered and local observation (.npz)")
    ap.add_argument("--envs-per-wave", type=int, default=0, choices=[0, 1, 2, 4, 8],
                    help="kernel tiling (0: the library default, 4); recorded in config")
    ap.add_argument("--bwd-envs-per-wave", type=int, default=0, choices=[0, 1, 2, 4, 8],
                    help="--mode grad: the backward launch's tiling (0: the forward's)")
    ap.add_argument("--specialize", type=int, default=1, choices=[0, 1],
                    help="0: the generic kernel instead of the reference scenes' specializations")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the multi-GPU path); gloo: ranks that share one GPU (tests), the "
                         "observation all-gather through host memory")
    ap.add_argument("--prng-layout", default="legacy", choices=["legacy", "partitionable"],
                    help="the jax.random threefry layout of the collider (cotix_params; JAX 0.4.x: legacy, "
                         "JAX >= 0.5: partitionable)")
    ap.add_argument("--lib", default=None, help="another build of libcotix_amd.so (A/B tooling); recorded in config")
    ap.add_argument("--key-helper", type=int, default=1, choices=[0, 1],
                    help="step launches of more than 16 steps with the key-window helper wave (the library "
                         "default, 1) or the step wave alone (0); recorded in config")
    ap.add_argument("--split-bwd", type=int, default=1, choices=[0, 1],
                    help="--mode grad: the RoboCup tape backward at two waves per env group (the library default, 1) "
                         "or one (0; other scenes always run one, DESIGN section 3); recorded in config")
    a = ap.parse_args()
    refuse_overrides()
    # the two-wave forms' library switches (read at the first launch)
    os.environ["COTIX_KEY_HELPER"] = str(a.key_helper)
    os.environ["COTIX_SPLIT_BWD"] = str(a.split_bwd)
    if a.lib:  # read by parallax_amd._ffi at import
        os.environ["COTIX_AMD_LIB"] = os.path.abspath(a.lib)
    return a


# environment variables the bench itself reads; any other COTIX_* variable
# could select another library or kernel behaviour behind the line's back
BENCH_ENV_OK = {"COTIX_BENCH_FORCE_DIST"}


def two_wave_forms():
    """The two-wave kernel forms this run allowed (--key-helper, --split-bwd):
    the key-window helper wave of step launches with more than one key
    window, the split tape backward (RoboCup; other scenes run MODE 4)."""
    return {"key_helper": int(os.environ.get("COTIX_KEY_HELPER", "1")),
            "split_bwd": int(os.environ.get("COTIX_SPLIT_BWD", "1"))}


def refuse_overrides():
    bad = sorted(k for k in os.environ if k.startswith("COTIX_") and k not in BENCH_ENV_OK)
    if bad:
        sys.exit("bench.py: refusing to run with COTIX_* overrides set (%s): kernel variants are bench "
                 "flags (--envs-per-wave, --specialize) and are recorded in the line" % ", ".join(bad))


# ---------------------------------------------------------------------------
# scenarios (global env ids [offset, offset+B) of a `total`-env run)
# ---------------------------------------------------------------------------
def make_scenario(pa, name, dev, B, offset=0, total=None, params=None):
    total = B if total is None else total
    sl = slice(offset, offset + B)
    if name == "robocup":
        return pa.RoboCupEnv(batch=B, device=dev, perturb=True, env_offset=offset, total_envs=total, params=params)
    if name == "box":
        return pa.BoxWorld(batch=B, device=dev, env_offset=offset, total_envs=total, params=params)
    tk = pa.random.split(pa.random.PRNGKey(0, dev), total, params)[sl].contiguous()
    ck = pa.random.split(pa.random.PRNGKey(1, dev), total, params)[sl].contiguous()
    return pa.LunarLander(key=tk, batch=B, device=dev, collider_keys=ck, params=params)


def bytes_per_env(name, nb):
    """Algorithmic HBM bytes per env per launch of BatchedEnv.step with
    autoreset: state in + out, key in + out, err in + out, the
    restart state read once, the restart counter in + out, the observation
    [nb][6] written by the kernel; LunarLander: + per-env terrain read."""
    b = nb * 6 * 4 * 2 + 16 + 8 + nb * 6 * 4 + 8 + nb * 6 * 4
    return b + (84 * 4 if name == "lunar" else 0)


WORKLOAD = {"robocup": "RoboCup (cotix/_robocup.py) %d envs/GPU",
            "lunar": "LunarLander (cotix/_lunar_lander.py) %d envs/GPU",
            "box": "BoxWorld (balls in a box, finite dynamics; not a reference scenario) %d envs/GPU"}


def obs_checksum(obs):
    """Position-weighted checksum of an observation tensor's bit patterns,
    exact in int64 (each product < 2^63, sums < 2^53): two weightings mod
    2^31 - 1, packed into one int64."""
    M = 2147483647
    v = (obs.contiguous().view(torch.int32).reshape(-1).to(torch.int64) & 0xFFFFFFFF) % M
    i = torch.arange(1, v.numel() + 1, dtype=torch.int64, device=v.device)
    a = ((v * (i * 48271 % M)) % M).sum() % M
    b = ((v * (i * 69621 % M)) % M).sum() % M
    return a * M + b


def timed_launches(fn, steps, warmup, separate=False):
    """`warmup` untimed calls, then `steps` calls bracketed by synchronize,
    HIP events around each call on the current stream.  Returns (wall s,
    mean event ms per call).  separate=True (short launches, K = 1): the wall
    pass runs with nothing else in the stream, as an RL loop calls it, and
    the event pass is `steps` more calls after it (event records between
    launches inflate the wall time of a 15 us launch by several us)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        if not separate:
            e0.record()
        fn()
        if not separate:
            e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if separate:
        for e0, e1 in evs:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
    return wall, sum(a.elapsed_time(b) for a, b in evs) / steps


def finite_stats(pa, scen, substeps, launches):
    """Diagnostics of a workload, outside any timed region: the same
    trajectory as the timed run (the fused kernel == one-step launches bit for
    bit, tests), stepped one driver step per launch with the state contract
    check after each step.  finite_env_fraction = fraction of env-steps that
    end on an all-finite state; restarts_per_env_step from the restart
    counters."""
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    w = env.world
    chk = torch.zeros(w.B, dtype=torch.int32, device=w.device)
    finite = torch.zeros((), dtype=torch.float64, device=w.device)
    n = substeps * launches
    for _ in range(n):
        env.step(1)
        chk.zero_()
        w.check_state(chk)
        finite += (chk == 0).sum()
    torch.cuda.synchronize()
    return {"finite_env_fraction": float(finite.item()) / (n * w.B),
            "restarts_per_env_step": float(env.resets.sum().item()) / (n * w.B),
            "sample": "%d envs x %d driver steps (one per launch + cotix_check_state)" % (w.B, n)}


def valu_roofline(scenario, B, substeps, launch_ms, warmup=None, layout="legacy"):
    """Primary roofline: VALU issue.  SQ_INSTS_VALU per launch from the
    committed rocprofv3 PMC pass of the same workload
    (profiles/latest_pmc_<scenario>.json, tools/gpu_round.sh) over the live
    launch time, against the chip's VALU issue peak.  HBM traffic per launch
    from the same pass (FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM")."""
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "latest_pmc_%s.json" % scenario)))
        c = pmc["config"]
        if not (c.get("envs_per_gpu") == B and c.get("substeps_per_launch") == substeps):
            return None
        if c.get("library") != library_build():  # counters of other kernel code: no frac
            return None
        if warmup is not None and pmc.get("warmup") != warmup:  # another stretch of the trajectory
            return None
        if c.get("prng_layout", "legacy") != layout:  # counters of the other PRNG layout's workload
            return None
        return {"valu_instr_per_launch": pmc["counters_per_launch"]["SQ_INSTS_VALU"],
                "traffic": pmc["hbm_bytes_per_launch_corrected"],
                "source": "profiles/%s_%s_summary.json" % (pmc["tag"], scenario),
                "valu_active_frac_of_wave_cycles": pmc["valu_active_frac_of_wave_cycles"],
                "wait_frac_of_wave_cycles": pmc.get("wait_frac_of_wave_cycles"),
                "stall": pmc.get("stall"),
                "kernel": pmc.get("kernel"),
                "pmc_avg_launch_ms": pmc["avg_launch_ns"] * 1e-6}
    except (OSError, KeyError, ValueError):
        return None


def library_build():
    """cotix_version() of the loaded libcotix_amd.so: it carries the build id
    (hash of the kernel sources and flags, __graft_entry__.build_id)."""
    from parallax_amd import _ffi
    return _ffi.lib.cotix_version().decode()


def roofline(scenario, B, substeps, launch_ms, nb, layout="legacy"):
    alg = bytes_per_env(scenario, nb) * B
    hbm = alg / (launch_ms * 1e-3) / 1e9
    out = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_WAVE_INSTR_S / 1e9, "unit": "G wave-instr/s",
           "frac": None, "traffic": None, "kernel": "step_kernel", "launch_ms": launch_ms,
           "hbm": {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm / HBM_PEAK_GBS,
                   "alg_bytes_per_launch": alg},
           "note": "VALU/latency-bound path (threefry integer rounds + f32 geometry, no dense contraction): "
                   "achieved = SQ_INSTS_VALU per launch / live launch time; peak = 256 CU x 4 SIMD x 2.4 GHz / "
                   "2 cycles per wave64 instruction (one wave per SIMD issues at most half of it); "
                   "hbm = algorithmic bytes / launch time, reported because north_star asks"}
    v = valu_roofline(scenario, B, substeps, launch_ms, layout=layout)
    if v is None:
        out["frac_note"] = ("no committed PMC pass (profiles/latest_pmc_%s.json) of this library build and "
                            "workload: frac left null rather than mixing counters of other code" % scenario)
    else:
        ach = v["valu_instr_per_launch"] / (launch_ms * 1e-3)
        out.update(achieved=ach / 1e9, frac=ach / VALU_PEAK_WAVE_INSTR_S, traffic=v["traffic"],
                   traffic_source=v["source"], valu_active_frac_of_wave_cycles=v["valu_active_frac_of_wave_cycles"],
                   wait_frac_of_wave_cycles=v["wait_frac_of_wave_cycles"], stall=v["stall"],
                   pmc_avg_launch_ms=v["pmc_avg_launch_ms"])
        if v.get("kernel"):  # the profiled kernel's full name (the RoboCup step: step_help_kernel)
            out["kernel"] = v["kernel"]
    return out


# ---------------------------------------------------------------------------
# CPU baselines (oracle C port: test infrastructure, timed here as the
# reported non-target baseline; never on the product path)
# ---------------------------------------------------------------------------
def host_cpu():
    """The host CPU the baselines ran on (model name from /proc/cpuinfo; the
    box's logical CPU count -- the threads used are each baseline's cores)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_logical_cpus": os.cpu_count()}


def cpu_baseline(scenario, seconds):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cotix_oracle import cport
    out = cport.time_baseline(scenario, seconds)
    out.update(host_cpu())
    return out


def cpu_config1(seconds=3.0):
    """Config 1 on ONE core: the C port runs the single LunarLander env
    (terrain PRNGKey(0), key chain from PRNGKey(0)) for 10,000 steps, repeated
    until `seconds` of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    lib = cport.load()
    bodies = P.lunar_lander_bodies(prng.PRNGKey(0))
    sc = cport.Scene(lib, bodies)
    geom = sc.geom[None].copy()
    d0 = np.ascontiguousarray(np.array([b.dyn() for b in bodies], np.float32)[:, :, None])
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds or n == 0:
        dyn, keys, err = d0.copy(), np.zeros((1, 2), np.uint32), np.zeros(1, np.uint32)
        sc.step(dyn, keys, err, 10000, cport.STAGES_LUNAR, geom, nthreads=1)
        n += 10000
    dt = time.perf_counter() - t0
    return dict({"value": n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
                 "sample": "%d x the 10,000-step trajectory, C oracle port, 1 thread, %.1f s" % (n // 10000, dt)},
                **host_cpu())


def cpu_baseline_grad(T, seconds):
    """Central finite differences (eps=1e-3) of the C oracle port (SURVEY.md
    8(d) config 5): 4T perturbed rollouts per env, OpenMP over all of them."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cotix_oracle import cport
    from cotix_oracle import physics as P
    lib = cport.load()
    sc = cport.Scene(lib, P.robocup_bodies())
    nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    w = np.zeros(30, np.float32)
    w[24] = 1.0

    def run(B):
        dyn, keys = cport.robocup_batch(B)
        acts = (np.random.default_rng(0).normal(size=(T, B, 2)) * 0.1).astype(np.float32)
        t0 = time.perf_counter()
        cport.fd_action_grad(sc, dyn, keys, acts, 4, w, cport.STAGES_ROBOCUP, eps=1e-3, nthreads=nthreads)
        return time.perf_counter() - t0

    B, dt = 8, run(8)
    while dt < 0.5 * seconds and B < 4096:
        B = int(min(4096, max(2 * B, B * seconds / max(dt, 1e-3))))
        dt = run(B)
    return dict({"value": B * T / dt, "unit": "env-steps/s (with d ret/d action)", "cores": nthreads, "kind": "port",
                 "sample": "%d RoboCup envs x %d-step rollout, gradient by central differences (%d perturbed "
                           "rollouts per env) of the C oracle port, OpenMP %d threads, %.1f s"
                           % (B, T, 4 * T, nthreads, dt)}, **host_cpu())


# ---------------------------------------------------------------------------
# secondary figures (rank 0, after the headline)
# ---------------------------------------------------------------------------
def sub_step(pa, dev, name, B, substeps, steps, warmup, key=None, layout="legacy"):
    """A secondary figure; `key` names its committed PMC pass
    (profiles/latest_pmc_<key>.json, default the scenario name), which must be
    of the same stretch of the trajectory (warm-up launches) for LunarLander,
    whose cost changes when the landers touch down.  layout: the scene's PRNG
    layout (cotix_params; the partitionable one is JAX >= 0.5's default)."""
    key = key or name
    params = pa.Params(prng_layout=layout)
    scen = make_scenario(pa, name, dev, B, params=params)
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    wall, ev_ms = timed_launches(lambda: env.step(substeps), steps, warmup, separate=substeps == 1)
    out = {"workload": WORKLOAD[name] % B, "substeps_per_launch": substeps, "launches": steps,
           "value": B * substeps * steps / wall, "unit": "env-steps/s", "launch_ms": ev_ms,
           "hbm_GBs": bytes_per_env(name, len(scen.bodies)) * B / (ev_ms * 1e-3) / 1e9, "prng_layout": layout,
           "kernel_variant": dict(scen.world.scene.variant(), **two_wave_forms())}
    v = valu_roofline(key, B, substeps, ev_ms, warmup if name == "lunar" else None, layout)
    if v is not None:  # the committed PMC pass of this workload (profiles/latest_pmc_<key>.json)
        out["valu"] = {"achieved": v["valu_instr_per_launch"] / (ev_ms * 1e-3) / 1e9,
                       "frac": v["valu_instr_per_launch"] / (ev_ms * 1e-3) / VALU_PEAK_WAVE_INSTR_S,
                       "unit": "G wave-instr/s", "traffic": v["traffic"], "source": v["source"]}
    out["driver_steps_timed"] = [warmup * substeps, (warmup + steps) * substeps]
    if name == "lunar":  # the regime: envs in which some body chose a contact partner over the next 8 steps
        tr = {}
        env.step(8, trace=tr)
        ch = tr["chosen"]  # [step][body][B], j* of body i (cotix/_colliders.py:274-295; i itself: none)
        own = torch.arange(ch.shape[1], device=ch.device, dtype=ch.dtype)[None, :, None]
        out["contact_env_fraction"] = float((ch != own).any(1).any(0).float().mean().item())
    out.update(finite_stats(pa, make_scenario(pa, name, dev, B, params=params), 1, 64))
    return out


def sub_grad(pa, dev, B, T, steps, warmup, scenario="robocup"):
    r = run_grad(pa, dev, B, T, steps, warmup, rank=0, world_size=1, scenario=scenario)
    out = {"workload": {"box": "BoxWorld %d envs, %d-step differentiable rollout, fwd + bwd (config 5 on a finite "
                                "scene)",
                        "lunar": "LunarLander %d envs settled on the terrain (after 2560 steps), %d-step "
                                 "differentiable rollout, fwd + bwd: gradients through GJK/EPA polygon contacts and "
                                 "the joints (lander x w.r.t. the lander's per-step dv)"}.get(
                scenario, "RoboCup %d envs, %d-step differentiable rollout, fwd + bwd (BASELINE config 5)") % (B, T),
           "value": r["value"], "unit": "env-steps/s with d(return)/d(action)", "fwd_ms": r["fwd_ms"],
           "bwd_ms": r["bwd_ms"], "finite_grad_env_fraction": r["finite"]}
    v = grad_valu({"box": "grad_box", "lunar": "grad_lunar"}.get(scenario, "grad"), B, T, r["fwd_ms"], r["bwd_ms"])
    if v is not None:
        out["valu"] = v
    return out


def sub_eval(pa, dev, B, nfe=4, wfe=16, steps=10, warmup=2):
    """AbstractEnvironment.eval (cotix/_envs.py:37-132) fused into one
    cotix_eval launch per call: RoboCup, a device judge (the goals as regions
    with their rewards, the ball's x-velocity as the reward rate, the error
    trip as done) and a device PD control on the ball, nfe x wfe env-steps
    at dt = 1e-2 from the same start state each call."""
    from parallax_amd import envs as E
    scen = make_scenario(pa, "robocup", dev, B)
    w = scen.world
    inf, ab = float("inf"), len(scen.bodies) - 1
    lo_y, hi_y = [-inf] * 6, [inf] * 6
    lo_b, hi_b = [-inf] * 6, [inf] * 6
    hi_y[0], lo_y[1], hi_y[1] = -4.5, -0.5, 0.5
    lo_b[0], lo_b[1], hi_b[1] = 4.5, -0.5, 0.5
    judge = E.LinearJudge(rate_w={6 * ab + 2: 0.1}, regions=[(ab, lo_y, hi_y, -1.0), (ab, lo_b, hi_b, 1.0)],
                          done_on_error=True)
    control = E.AffineControl(body=ab, gain=[[0, 0, 0.1, 0, 0, 0], [0, 0, 0, 0.1, 0, 0]],
                              target=[[0, 0, 2.0, 0, 0, 0], [0] * 6])
    env = E.AbstractEnvironment(E.PhysicsWorld(w, scen.stages), E.WorldState(w.dyn.clone(), w.keys.clone(),
                                                                            w.err.clone()), control, judge)
    assert env.fused()
    period = nfe * wfe * 1e-2
    state = {}
    wall, ev_ms = timed_launches(lambda: state.update(r=env.eval(period, nfe, wfe)[1]), steps, warmup)
    return {"workload": "RoboCup %d envs, AbstractEnvironment.eval with a device judge and control, %d NFEs x %d "
                        "env-steps in one launch (cotix_eval)" % (B, nfe, wfe),
            "value": B * nfe * wfe * steps / wall, "unit": "env-steps/s", "launch_ms": ev_ms,
            "finite_reward_fraction": float(torch.isfinite(state["r"]).float().mean().item())}


def sub_config1(pa, dev):
    """BASELINE config 1: one LunarLander env (PRNGKey(0) terrain and key
    chain), 10,000 driver steps in one launch (latency-bound: one wave)."""
    ll = pa.LunarLander(batch=1, device=dev)
    dyn0, keys0 = ll.world.dyn.clone(), ll.world.keys.clone()

    def run():
        ll.world.dyn.copy_(dyn0)
        ll.world.keys.copy_(keys0)
        ll.world.err.zero_()
        ll.world.step(10000, 1e-2, ll.stages)

    wall, ev_ms = timed_launches(run, 3, 1)
    return {"workload": "LunarLander single env, 10,000 steps in one launch (BASELINE config 1)",
            "value": 10000 / (ev_ms * 1e-3), "unit": "env-steps/s", "ms_per_10000_steps": ev_ms,
            "cpu_1core": cpu_config1()}


# ---------------------------------------------------------------------------
# headline
# ---------------------------------------------------------------------------
def init_dist(force=False, backend="nccl"):
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # COTIX_BENCH_FORCE_DIST=1: the collective path at world size 1 too (needs
    # RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT, as torchrun sets them)
    if world_size > 1 or force:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    return dist, rank, world_size, torch.device("cuda", local_rank)


def main():
    a = parse()
    if a.mode == "grad":
        return main_grad(a)
    dist, rank, world_size, dev = init_dist(os.environ.get("COTIX_BENCH_FORCE_DIST") == "1", a.dist_backend)
    import parallax_amd as pa
    gloo = dist is not None and a.dist_backend == "gloo"
    cdev = torch.device("cpu") if gloo else dev  # where the collectives' tensors live

    B = a.envs
    params = pa.Params(prng_layout=a.prng_layout)
    scen = make_scenario(pa, a.scenario, dev, B, rank * B, world_size * B, params)
    scen.world.set_variant(a.envs_per_wave, bool(a.specialize))
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    nbody = len(scen.bodies)
    # observation all-gather, double-buffered and asynchronous: the RCCL
    # collective of launch i runs on its own stream while launch i+1 computes;
    # a buffer is rewritten only after the collective that read it is done
    obs_all = [torch.empty(world_size * B, nbody, 6, device=cdev) for _ in range(2)] if dist else None
    obs_local = [torch.empty(B, nbody, 6, device=dev) for _ in range(2)] if dist else None
    pending = [None, None]
    launches = [0]
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]

    def one_step(i=None):
        k = launches[0] % 2
        if dist is not None and pending[k] is not None:
            pending[k].wait()  # the current stream waits for the collective that read buffer k
        if i is not None:
            evs[i][0].record()
        # the step kernel writes the observation straight into the send buffer
        env.step(a.substeps, obs_out=obs_local[k] if dist is not None else None)
        if i is not None:
            evs[i][1].record()
        if dist is not None:  # north star: RCCL all-gather of the observation tensor
            launches[0] += 1
            send = obs_local[k].cpu() if gloo else obs_local[k]
            pending[k] = dist.all_gather_into_tensor(obs_all[k], send, async_op=True)

    def drain():
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    for _ in range(a.warmup):
        one_step()
    drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        one_step(i)
    drain()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs)
    tmax = torch.tensor([wall], device=cdev, dtype=torch.float64)
    if dist:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    wall = float(tmax.item())
    resets = int(env.resets.sum().item())
    gather = None
    if dist is not None:
        # every slice of the gathered tensor must be its owner's local observation:
        # each rank publishes a checksum of its own obs bits, every rank checks all slices
        last = (launches[0] - 1) % 2
        local = env.observation()
        sums = torch.zeros(world_size, dtype=torch.int64, device=cdev)
        sums[rank] = obs_checksum(local).to(cdev)
        dist.all_reduce(sums)
        got = torch.stack([obs_checksum(obs_all[last][r * B:(r + 1) * B]) for r in range(world_size)]).to(cdev)
        bad = torch.tensor([int((got != sums).sum().item())], dtype=torch.int64, device=cdev)
        dist.all_reduce(bad)
        gather = "ok (%d slices checked on every rank)" % world_size if int(bad.item()) == 0 else "MISMATCH"
        if a.dump_gather and rank == 0:
            np.savez(a.dump_gather, gathered=obs_all[last].cpu().numpy(), local=local.cpu().numpy(),
                     dyn=env.world.dyn.cpu().numpy())

    launch_ms = ev_ms / a.steps
    env_steps = B * a.substeps * a.steps * world_size
    out = {
        "metric": "env steps/sec (whole node), RoboCup 4096 envs/GPU, at 1/2/4/8 MI355X"
        if a.scenario == "robocup" else "env steps/sec (whole node), %s" % (WORKLOAD[a.scenario] % B),
        "value": env_steps / wall,
        "unit": "env-steps/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (reference scenario constructors; per-env perturbation/terrain from threefry keys "
                "of the global env id)",
        "config": {
            "workload": WORKLOAD[a.scenario] % B,
            "envs_per_gpu": B,
            "substeps_per_launch": a.substeps,
            "autoreset_on_error": True,
            "library": library_build(),
            "library_path": a.lib or "parallax_amd/_lib/libcotix_amd.so",
            "kernel_variant": dict(scen.world.scene.variant(), **two_wave_forms()),
            "prng_layout": a.prng_layout,
            "episode_restarts": resets,
            "restarts_per_env_step": resets / (B * a.substeps * (a.steps + a.warmup)),
            "parallelism": "dp%d (independent env shards by global env id, %s obs all-gather)"
                           % (world_size, "gloo (host)" if gloo else "RCCL"),
        },
        "roofline": roofline(a.scenario, B, a.substeps, launch_ms, nbody, a.prng_layout),
    }
    if gather is not None:
        out["config"]["obs_all_gather_check"] = gather
    # the CPU baseline and the secondary figures: one-GPU runs only (an N-GPU
    # line carries the headline; the other ranks would idle in the barrier)
    single = world_size == 1
    if rank == 0 and single and a.extras == "auto":  # (the headline's own workload: its PRNG layout)
        out["workload_stats"] = finite_stats(pa, make_scenario(pa, a.scenario, dev, B, params=params), 1, 64)
        out["workload_stats"]["prng_layout"] = a.prng_layout
    if rank == 0 and single and a.extras == "auto" and a.scenario == "robocup":
        out["k1"] = sub_step(pa, dev, "robocup", B, 1, 2000, 50)
        # the headline scene in JAX >= 0.5's partitionable threefry layout (the
        # reference pins no JAX version, pyproject.toml:16)
        out["robocup_partitionable"] = sub_step(pa, dev, "robocup", B, a.substeps, 10, 2, key="robocup_part",
                                                layout="partitionable")
        out["finite_scene"] = sub_step(pa, dev, "box", B, a.substeps, 10, 2)
        out["lunar"] = sub_step(pa, dev, "lunar", B, a.substeps, 10, 2)  # airborne: driver steps 128-768
        # the landers settled on the terrain (first touch-down ~770, a bounce, settled from
        # ~2500: tools/ll_regime.py, profiles/r03_ll_regime.json): driver steps 2560-3200
        out["lunar_contact"] = sub_step(pa, dev, "lunar", B, a.substeps, 10, 40, key="lunar_contact")
        out["grad"] = sub_grad(pa, dev, B, 64, 5, 1)
        out["grad_box"] = sub_grad(pa, dev, B, 64, 5, 1, scenario="box")
        out["grad_lunar"] = sub_grad(pa, dev, B, 64, 5, 1, scenario="lunar")
        out["eval"] = sub_eval(pa, dev, B)
        out["config1"] = sub_config1(pa, dev)
    # the CPU baseline last: its OpenMP threads must not compete with the
    # host thread that launches the GPU figures (the K = 1 loop is launch-bound)
    if rank == 0 and single and a.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline(a.scenario if a.scenario != "box" else "robocup", a.cpu_seconds)
        if a.extras == "auto" and a.scenario == "robocup":  # the sub-figures' own baselines (configs 2 and 5)
            out["lunar"]["cpu_baseline"] = cpu_baseline("lunar", a.cpu_seconds / 2)
            out["grad"]["cpu_baseline"] = cpu_baseline_grad(64, a.cpu_seconds / 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# config 5 as its own line
# ---------------------------------------------------------------------------
def run_grad(pa, dev, B, T, steps, warmup, rank, world_size, dist=None, scenario="robocup", tiling=(0, 1, 0)):
    """Config 5: forward (cotix_rollout) + backward (cotix_rollout_backward)
    of a T-step rollout, d(sum_t x of the action body)/d(per-step dv of it).
    scenario "box": the same on the box world (finite dynamics), whose
    gradients are finite -- RoboCup's degenerate reference scene makes most
    of its envs' gradients NaN."""
    stages, ab = pa._ffi.STAGES_ROBOCUP, None
    if scenario == "box":
        scen = pa.BoxWorld(batch=B, device=dev, env_offset=rank * B, total_envs=world_size * B)
    elif scenario == "lunar":
        # LunarLander settled on its terrain (driver steps 2560+, the lunar_contact
        # regime): GJK/EPA polygon contacts and the joints every step
        scen = pa.LunarLander(batch=B, device=dev)
        stages, ab = pa._ffi.STAGES_LUNAR | pa._ffi.STAGE_BROADPHASE, 0
        for _ in range(40):
            scen.world.step(64, 1e-2, stages)
    else:
        scen = pa.RoboCupEnv(batch=B, device=dev, perturb=True, env_offset=rank * B, total_envs=world_size * B)
    world = scen.world
    nb = len(world.bodies)
    ab = nb - 1 if ab is None else ab
    ew, spec, bwd_ew = tiling  # (--envs-per-wave, --specialize, --bwd-envs-per-wave)
    world.set_variant(ew, bool(spec))
    variant = world.scene.variant()
    dyn0, keys0 = world.dyn.clone(), world.keys.clone()
    gen = torch.Generator(device="cpu").manual_seed(1234 + rank)
    actions = (torch.randn(T, B, 2, generator=gen) * 0.1).to(dev)  # ball dv ~ N(0, 0.1^2)
    w = pa.rollout.ball_x_weights(nb, ab)  # RoboCup: the ball (body 4); box world: the last ball; LL: the lander
    evf = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    evb = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    state = {}

    def one_step(i=None):
        world.dyn.copy_(dyn0)
        world.keys.copy_(keys0)
        world.err.zero_()
        if i is not None:
            evf[i][0].record()
        ret, saved = pa.rollout_forward(world, actions, ab, w, stages=stages)
        if i is not None:
            evf[i][1].record()
            evb[i][0].record()
        if bwd_ew:
            world.set_variant(bwd_ew, bool(spec))
        ga, _ = pa.rollout_backward(world, saved)
        if bwd_ew:
            world.set_variant(ew, bool(spec))
        if i is not None:
            evb[i][1].record()
        state["ret"], state["ga"] = ret, ga

    for _ in range(warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one_step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tmax = torch.tensor([wall], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    wall = float(tmax.item())
    ga = state["ga"]
    return {"value": B * T * steps * world_size / wall, "wall": wall, "variant": variant,
            "fwd_ms": sum(e0.elapsed_time(e1) for e0, e1 in evf) / steps,
            "bwd_ms": sum(e0.elapsed_time(e1) for e0, e1 in evb) / steps,
            "finite": float(torch.isfinite(ga).all(dim=2).all(dim=0).float().mean().item()),
            "tape_words": int(pa._ffi.lib.cotix_rollout_tape_words(world.scene.handle))}


def grad_valu(key, B, T, fwd_ms, bwd_ms):
    """VALU fractions of the rollout's forward (MODE 1) and backward (MODE 2)
    kernels from the committed PMC pass of this build and workload
    (profiles/latest_pmc_<key>.json, per-kernel counters), or None."""
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "latest_pmc_%s.json" % key)))
        c = pmc["config"]
        if not (c.get("envs_per_gpu") == B and c.get("rollout_steps") == T and pmc.get("library") == library_build()):
            return None
        out = {}
        for part, ms in (("fwd", fwd_ms), ("bwd", bwd_ms)):
            k = pmc["kernels"][part]
            ach = k["counters_per_launch"]["SQ_INSTS_VALU"] / (ms * 1e-3)
            out[part] = {"achieved": ach / 1e9, "frac": ach / VALU_PEAK_WAVE_INSTR_S, "unit": "G wave-instr/s",
                         "kernel": k["kernel"], "pmc_avg_launch_ms": k["avg_launch_ns"] * 1e-6,
                         "valu_active_frac_of_wave_cycles": k["valu_active_frac_of_wave_cycles"],
                         "traffic": k["hbm_bytes_per_launch_corrected"]}
        out["source"] = "profiles/%s_%s_summary.json" % (pmc["tag"], key)
        return out
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def main_grad(a):
    """BASELINE config 5: differentiable RoboCup rollout, forward + backward
    (--scenario box: the box world)."""
    dist, rank, world_size, dev = init_dist()
    import parallax_amd as pa
    B, T = a.envs, a.substeps
    box, lunar = a.scenario == "box", a.scenario == "lunar"
    r = run_grad(pa, dev, B, T, a.steps, a.warmup, rank, world_size, dist,
                 "box" if box else ("lunar" if lunar else "robocup"),
                 (a.envs_per_wave, a.specialize, a.bwd_envs_per_wave))
    nb = 7 if box else (4 if lunar else 5)
    key = "grad_box" if box else ("grad_lunar" if lunar else "grad")
    # algorithmic HBM bytes per env-step.  Backward: saved state (nb x 6 f32)
    # + key (2 u32) + action (2 f32) + the whole decision tape (tape_words
    # u32: per body the resolution words; analytic scenes the resolution
    # records, polygon scenes EPA's recorded edge per distinct contact --
    # counted in full, an upper bound where a contact's edge is read only
    # when it was resolved) read, grad_action (2 f32) written.  Forward:
    # action read, saved state + key + the tape written (the state itself is
    # read and written once per launch).
    tw = r["tape_words"]
    bwd_bytes = (nb * 6 * 4 + 8 + 8 + tw * 4 + 8) * B * T
    fwd_bytes = (8 + nb * 6 * 4 + 8 + tw * 4) * B * T + (nb * 6 * 4 + 8 + 4) * 2 * B
    achieved = bwd_bytes / (r["bwd_ms"] * 1e-3) / 1e9
    out = {
        "metric": "differentiable %d-step %s rollout, %d envs/GPU: env-steps/s with d(return)/d(action)"
                  % (T, "box-world" if box else ("LunarLander" if lunar else "RoboCup"), B),
        "value": r["value"],
        "unit": "env-steps/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": r["wall"] * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (%s; actions N(0, 0.1^2) per step)"
                % ("box world, per-env random balls" if box else
                   ("LunarLander settled on its terrain after 2560 steps" if lunar else
                    "RoboCup scene, per-env ball perturbation")),
        "config": {
            "workload": ("BoxWorld %d envs/GPU, %d-step rollout, grad of sum_t x of the last ball w.r.t. its "
                         "per-step dv (config 5 on a finite scene)" if box else
                         ("LunarLander %d envs/GPU settled on the terrain, %d-step rollout, grad of sum_t lander "
                          "x w.r.t. the lander's per-step dv (GJK/EPA contacts and joints)" if lunar else
                          "RoboCup (cotix/_robocup.py) %d envs/GPU, %d-step rollout, grad of sum_t ball x "
                          "w.r.t. per-step ball dv (BASELINE config 5)")) % (B, T),
            "envs_per_gpu": B,
            "rollout_steps": T,
            "fwd_ms": r["fwd_ms"],
            "bwd_ms": r["bwd_ms"],
            "finite_grad_env_fraction": r["finite"],
            "library": library_build(),
            "kernel_variant": dict(r["variant"], **two_wave_forms()),
            "parallelism": "dp%d (independent env shards)" % world_size,
        },
        "roofline": {
            "bound": "valu",
            "achieved": None,
            "peak": VALU_PEAK_WAVE_INSTR_S / 1e9,
            "unit": "G wave-instr/s",
            "frac": None,
            "traffic": None,
            "kernel": "step_kernel<4,F,4> (backward from the forward's tape)",
            "launch_ms": r["bwd_ms"],
            "hbm": {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                    "alg_bytes_per_launch": bwd_bytes, "tape_words_per_env_step": tw,
                    "fwd_alg_bytes_per_launch": fwd_bytes,
                    "fwd_achieved": fwd_bytes / (r["fwd_ms"] * 1e-3) / 1e9},
            "note": "VALU/latency-bound (per step: Euler, world parts, the tape's resolutions, the VJP chain)",
        },
    }
    v = grad_valu(key, B, T, r["fwd_ms"], r["bwd_ms"])
    if v is None:
        out["roofline"]["frac_note"] = "no committed PMC pass of this build and workload: frac left null"
    else:
        out["roofline"].update(achieved=v["bwd"]["achieved"], frac=v["bwd"]["frac"], traffic=v["bwd"]["traffic"],
                               fwd=v["fwd"], traffic_source=v["source"])
    if rank == 0 and world_size == 1 and a.cpu_baseline == "auto" and not lunar:
        out["cpu_baseline"] = cpu_baseline_grad(T, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
