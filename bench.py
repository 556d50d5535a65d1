"""Benchmark: RoboCup, 4096 envs per GPU, env-steps/s (BASELINE.json metric).

One bench "step" = one launch of the fused HIP step kernel advancing every
env by --substeps driver steps (examples/test_viz.py:61-69: Euler ->
RandomizedCollider -> identity constraint pass -> key split), with episode
restarts on the reference's error_if trip (DESIGN.md "Benchmark").  Inputs are
resident in HBM before the timed region.  value = envs * substeps * steps *
n_gpus / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W --substeps S --scenario robocup|lunar]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)

--mode grad (BASELINE config 5): one bench step = a differentiable --substeps
(64) step RoboCup rollout from a fixed start state, forward (cotix_rollout)
+ backward (cotix_rollout_backward) -> d(sum_t ball x)/d(action) for every
env; value = envs * substeps * steps * n_gpus / wall (env-steps with
gradient per second).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--substeps", type=int, default=64)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--scenario", default="robocup", choices=["robocup", "lunar"])
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--mode", default="step", choices=["step", "grad"])
    return ap.parse_args()


def cpu_baseline(scenario, seconds):
    """Oracle port timed on this host (bounded sample).  Prefers the C port
    (oracle/build/libcotix_oracle.so, OpenMP over envs), else the Python
    oracle on one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        from cotix_oracle import cport
        return cport.time_baseline(scenario, seconds)
    except (ImportError, OSError):
        pass
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    d0 = prng.gjk_initial_direction()
    mk = P.robocup_bodies if scenario == "robocup" else (lambda: P.lunar_lander_bodies(prng.PRNGKey(0)))
    step = P.robocup_step if scenario == "robocup" else P.lunar_lander_step
    n, t0 = 0, time.perf_counter()
    bodies, key = mk(), prng.PRNGKey(0)
    while time.perf_counter() - t0 < seconds:
        err = G.ErrorFlag()
        bodies, key = step(bodies, key, d0, err)
        if err.bits:
            bodies = mk()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "%d sequential env-steps of one %s env (python oracle, autoreset), %.1f s" % (n, scenario, dt)}


def cpu_baseline_grad(T, seconds):
    """Central finite differences (eps=1e-3) of the C oracle port (SURVEY.md
    8(d) config 5): 4T perturbed rollouts per env, OpenMP over all of them.
    Bounded sample sized from a short probe to ~`seconds`."""
    import numpy as np
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
    while dt < 0.5 * seconds and B < 4096:  # grow the sample to ~`seconds` of CPU work
        B = int(min(4096, max(2 * B, B * seconds / max(dt, 1e-3))))
        dt = run(B)
    return {"value": B * T / dt, "unit": "env-steps/s (with d ret/d action)", "cores": nthreads, "kind": "port",
            "sample": "%d RoboCup envs x %d-step rollout, gradient by central differences (%d perturbed rollouts "
                      "per env) of the C oracle port, OpenMP %d threads, %.1f s" % (B, T, 4 * T, nthreads, dt)}


def main():
    a = parse()
    if a.mode == "grad":
        return main_grad(a)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # COTIX_BENCH_FORCE_DIST=1: the collective path at world size 1 too (tests the RCCL code on one GPU)
    if world_size > 1 or os.environ.get("COTIX_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    import parallax_amd as pa

    B = a.envs
    # global env ids [rank*B, (rank+1)*B): keys split(PRNGKey(seed), B*world)[ids]
    if a.scenario == "robocup":
        keys = pa.random.split(pa.random.PRNGKey(3, dev), B * world_size)[rank * B:(rank + 1) * B].contiguous()
        scen = pa.RoboCupEnv(batch=B, device=dev, keys=keys, perturb=True)
        bytes_per_env = 5 * 6 * 4 * 2 + 16 + 8
    else:
        tk = pa.random.split(pa.random.PRNGKey(0, dev), B * world_size)[rank * B:(rank + 1) * B].contiguous()
        ck = pa.random.split(pa.random.PRNGKey(1, dev), B * world_size)[rank * B:(rank + 1) * B].contiguous()
        scen = pa.LunarLander(key=tk, batch=B, device=dev, collider_keys=ck)
        bytes_per_env = 4 * 6 * 4 * 2 + 16 + 8 + 84 * 4
    env = pa.BatchedEnv(scen, autoreset=True)
    env.reset()
    # observation all-gather, double-buffered and asynchronous: the RCCL
    # collective of launch i runs on its own stream while launch i+1 computes;
    # a buffer is rewritten only after the collective that read it is done
    nbody = len(scen.bodies)
    obs_all = [torch.empty(world_size * B, nbody, 6, device=dev) for _ in range(2)] if dist else None
    obs_local = [torch.empty(B, nbody, 6, device=dev) for _ in range(2)] if dist else None
    pending = [None, None]
    launches = [0]

    # HIP events around every step-kernel launch, on the stream it runs on
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]

    def one_step(i=None):
        if i is not None:
            evs[i][0].record()
        env.step(a.substeps)
        if i is not None:
            evs[i][1].record()
        if dist is not None:  # north star: RCCL all-gather of the observation tensor
            k = launches[0] % 2
            launches[0] += 1
            if pending[k] is not None:
                pending[k].wait()  # the current stream waits for the collective that read buffer k
            env.observation(obs_local[k])
            pending[k] = dist.all_gather_into_tensor(obs_all[k], obs_local[k], async_op=True)

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
    tmax = torch.tensor([wall], device=dev, dtype=torch.float64)
    if dist:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    wall = float(tmax.item())
    resets = int(env.resets.sum().item())

    # per-launch kernel time from HIP events on the launch stream (timed region)
    launch_ms = ev_ms / a.steps
    alg_bytes = bytes_per_env * B  # HBM bytes one launch must move (state in + out)
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
    env_steps = B * a.substeps * a.steps * world_size
    out = {
        "metric": "env steps/sec (whole node), RoboCup 4096 envs/GPU, at 1/2/4/8 MI355X"
        if a.scenario == "robocup" else "env steps/sec (whole node), LunarLander 4096 envs/GPU",
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
        "data": "synthetic (reference scenario constructors; per-env perturbation/terrain from threefry keys)",
        "config": {
            "workload": ("RoboCup (cotix/_robocup.py) %d envs/GPU" if a.scenario == "robocup"
                         else "LunarLander (cotix/_lunar_lander.py) %d envs/GPU") % B,
            "envs_per_gpu": B,
            "substeps_per_launch": a.substeps,
            "autoreset_on_error": True,
            "episode_restarts": resets,
            "parallelism": "dp%d (independent env shards, RCCL obs all-gather)" % world_size,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "step_kernel",
            "launch_ms": launch_ms,
            "alg_bytes_per_launch": alg_bytes,
            "note": "VALU/latency-bound path (no dense contraction); HBM figure reported because north_star asks",
        },
    }
    # HBM traffic per launch from the committed rocprofv3 PMC pass of the same
    # workload (profiles/latest_pmc_<scenario>.json, tools/gpu_round.sh);
    # FETCH_SIZE doubled per MI355X_MICROARCH.md "HBM" (gfx950 reports half
    # the bytes).  The same pass gives the VALU issue fraction -- the bound
    # that actually limits this path.
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "latest_pmc_%s.json" % a.scenario)))
        c = pmc["config"]
        if (c.get("envs_per_gpu") == B and c.get("substeps_per_launch") == a.substeps
                and c.get("workload", "").split()[0] == out["config"]["workload"].split()[0]):
            out["roofline"]["traffic"] = pmc["hbm_bytes_per_launch_corrected"]
            out["roofline"]["traffic_source"] = "profiles/%s_%s_summary.json" % (pmc["tag"], a.scenario)
            out["roofline"]["valu_issue_frac"] = pmc["valu_active_frac_of_wave_cycles"]
    except (OSError, KeyError, ValueError):
        pass
    if rank == 0 and a.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline(a.scenario, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def main_grad(a):
    """BASELINE config 5: differentiable RoboCup rollout, forward + backward."""
    import numpy as np
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    import parallax_amd as pa
    B, T = a.envs, a.substeps
    keys = pa.random.split(pa.random.PRNGKey(3, dev), B * world_size)[rank * B:(rank + 1) * B].contiguous()
    scen = pa.RoboCupEnv(batch=B, device=dev, keys=keys, perturb=True)
    world = scen.world
    dyn0, keys0 = world.dyn.clone(), world.keys.clone()
    gen = torch.Generator(device="cpu").manual_seed(1234 + rank)
    actions = (torch.randn(T, B, 2, generator=gen) * 0.1).to(dev)  # ball dv ~ N(0, 0.1^2)
    w = pa.rollout.ball_x_weights(5, 4)
    evf = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    evb = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    state = {}

    def one_step(i=None):
        world.dyn.copy_(dyn0)
        world.keys.copy_(keys0)
        world.err.zero_()
        if i is not None:
            evf[i][0].record()
        ret, saved = pa.rollout_forward(world, actions, 4, w)
        if i is not None:
            evf[i][1].record()
            evb[i][0].record()
        ga, _ = pa.rollout_backward(world, saved)
        if i is not None:
            evb[i][1].record()
        state["ret"], state["ga"] = ret, ga

    for _ in range(a.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
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
    fwd_ms = sum(e0.elapsed_time(e1) for e0, e1 in evf) / a.steps
    bwd_ms = sum(e0.elapsed_time(e1) for e0, e1 in evb) / a.steps
    ga = state["ga"]
    finite = float(torch.isfinite(ga).all(dim=2).all(dim=0).float().mean().item())
    # algorithmic HBM bytes of the backward launch per env-step: saved state
    # (5x6 f32) + key (2 u32) + action (2 f32) read, grad_action (2 f32) written
    bwd_bytes = (5 * 6 * 4 + 8 + 8 + 8) * B * T
    achieved = bwd_bytes / (bwd_ms * 1e-3) / 1e9
    out = {
        "metric": "differentiable 64-step RoboCup rollout, 4096 envs/GPU: env-steps/s with d(return)/d(action)",
        "value": B * T * a.steps * world_size / wall,
        "unit": "env-steps/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (RoboCup scene, per-env ball perturbation; actions N(0, 0.1^2) per step)",
        "config": {
            "workload": "RoboCup (cotix/_robocup.py) %d envs/GPU, %d-step rollout, grad of sum_t ball x "
                        "w.r.t. per-step ball dv (BASELINE config 5)" % (B, T),
            "envs_per_gpu": B,
            "rollout_steps": T,
            "fwd_ms": fwd_ms,
            "bwd_ms": bwd_ms,
            "finite_grad_env_fraction": finite,
            "parallelism": "dp%d (independent env shards)" % world_size,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "step_kernel<4,1,true> (backward re-play)",
            "launch_ms": bwd_ms,
            "alg_bytes_per_launch": bwd_bytes,
            "note": "VALU/latency-bound (the backward re-plays each step's forward); HBM figure for completeness",
        },
    }
    if rank == 0 and a.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline_grad(T, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
