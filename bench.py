"""Benchmark: RoboCup, 4096 envs per GPU, env-steps/s (BASELINE.json metric).

One bench "step" = one launch of the fused HIP step kernel advancing every
env by --substeps driver steps (examples/test_viz.py:61-69: Euler ->
RandomizedCollider -> identity constraint pass -> key split), with episode
restarts on the reference's error_if trip (DESIGN.md "Benchmark").  Inputs are
resident in HBM before the timed region.  value = envs * substeps * steps *
n_gpus / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W --substeps S --scenario robocup|lunar]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)
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


def main():
    a = parse()
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
    obs_all = torch.empty(world_size * B, len(scen.bodies), 6, device=dev) if dist else None

    def one_step():
        env.step(a.substeps)
        if dist is not None:  # north star: RCCL all-gather of the observation tensor
            dist.all_gather_into_tensor(obs_all, env.observation().contiguous())

    for _ in range(a.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        one_step()
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
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
    # workload (profiles/latest_pmc.json, tools/gpu_profile.sh); FETCH_SIZE
    # doubled per MI355X_MICROARCH.md "HBM" (gfx950 reports half the bytes).
    try:
        pmc = json.load(open(os.path.join(ROOT, "profiles", "latest_pmc.json")))
        c = pmc["config"]
        if (c.get("envs_per_gpu") == B and c.get("substeps_per_launch") == a.substeps
                and c.get("workload", "").split()[0] == out["config"]["workload"].split()[0]):
            out["roofline"]["traffic"] = pmc["hbm_bytes_per_launch_corrected"]
            out["roofline"]["traffic_source"] = "profiles/%s_summary.json" % pmc["tag"]
    except (OSError, KeyError, ValueError):
        pass
    if rank == 0 and a.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline(a.scenario, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
