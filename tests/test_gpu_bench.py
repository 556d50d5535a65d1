"""bench.py's multi-GPU code path on the one GPU of the box: the RCCL
("nccl") process group, the asynchronous double-buffered all-gather of the
observation tensor and the barrier / max-over-ranks timing, in a fresh child
process that initialises the GPU itself (WORLD_SIZE=1 plus the torchrun
variables, COTIX_BENCH_FORCE_DIST=1)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_rccl_path_single_rank(tmp_path):
    dump = str(tmp_path / "gather.npz")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), COTIX_BENCH_FORCE_DIST="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--substeps", "8", "--cpu-baseline", "off", "--extras", "off", "--dump-gather", dump],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["obs_all_gather_check"].startswith("ok")
    assert line["n_gpus"] == 1 and line["value"] > 0
    d = np.load(dump)
    # the gathered tensor == cotix_observe of the local state == the SoA state transposed
    assert np.array_equal(d["gathered"].view(np.uint32), d["local"].view(np.uint32))
    assert np.array_equal(d["local"].view(np.uint32), d["dyn"].transpose(2, 0, 1).view(np.uint32))


def _reference_obs(B, substeps, launches):
    """The single-rank run over all B envs of the bench workload: the
    observation after `launches` BatchedEnv.step(substeps) launches."""
    import torch
    sys.path.insert(0, ROOT)
    import parallax_amd as pa
    env = pa.BatchedEnv(pa.RoboCupEnv(batch=B, device="cuda", perturb=True), autoreset=True)
    env.reset()
    for _ in range(launches):
        env.step(substeps)
    torch.cuda.synchronize()
    return env.observation().cpu().numpy()


def test_bench_two_ranks_one_gpu(tmp_path):
    """bench.py's multi-rank path against the real kernel: two fresh child
    processes, ranks 0 and 1 of WORLD_SIZE=2, both on the box's one GPU
    (--dist-backend gloo: the observation all-gather through host memory,
    RCCL keeps one rank per device).  Each rank builds its shard from its
    global env ids; the barrier / max-over-ranks timing and the every-slice
    gather check run for real, and the gathered tensor equals a single-rank
    run over all 2B envs bit for bit."""
    B, sub, steps, warm = 256, 8, 2, 1
    dump = str(tmp_path / "gather.npz")
    port = str(_free_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--envs", str(B), "--steps",
                                       str(steps), "--warmup", str(warm), "--substeps", str(sub), "--cpu-baseline",
                                       "off", "--extras", "off", "--dist-backend", "gloo", "--dump-gather", dump],
                                      env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    line = json.loads(outs[0][0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["obs_all_gather_check"] == "ok (2 slices checked on every rank)"
    assert line["value"] > 0
    d = np.load(dump)
    want = _reference_obs(2 * B, sub, steps + warm)
    assert d["gathered"].shape == want.shape
    assert np.array_equal(d["gathered"].view(np.uint32), want.view(np.uint32))
    assert np.array_equal(d["local"].view(np.uint32), want[:B].view(np.uint32))  # rank 0's slice
