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
