"""Multi-GPU path on CPU: world_size-2 gloo.  Each rank owns a contiguous env
range (global ids rank*B .. rank*B+B-1, collider keys from ONE global
split, as bench.py does), steps it with the fused kernel's logic (host
emulation, tests/emu) and all-gathers the observation tensor (the north
star's RCCL all-gather, here over gloo).  The gathered result must equal a
single-rank run over all envs bit for bit: envs are independent, so the
sharding needs no data-path collective."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
B_LOCAL, T, WORLD = 8, 6, 2


def _setup_paths():
    for p in (os.path.join(HERE, "emu"), os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _initial_state(B):
    """RoboCup reset state for B envs (ball perturbed per env) + global keys."""
    _setup_paths()
    import make_golden as mg
    from cotix_oracle import physics as P
    from cotix_oracle import prng
    pert = mg.robocup_perturb(B)
    dyn = np.zeros((5, 6, B), np.float32)
    for e in range(B):
        d = [b.dyn() for b in P.robocup_bodies()]
        d[4] = list(pert[e])
        dyn[:, :, e] = np.array(d, np.float32)
    keys = np.ascontiguousarray(prng.split(prng.PRNGKey(3), B)).astype(np.uint32)
    return dyn, keys


def _run(dyn, keys):
    _setup_paths()
    import emu
    from cotix_oracle import physics as P
    lib = emu.load()
    h, geom = emu.oracle_scene(lib, P.robocup_bodies())
    dyn = np.ascontiguousarray(dyn)
    keys = np.ascontiguousarray(keys)
    err = np.zeros(dyn.shape[2], np.uint32)
    emu.step(lib, h, dyn, keys, err, geom, 0, T, 1 | 4 | 16)
    return dyn, keys, err


def _worker(rank, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    dyn_all, keys_all = _initial_state(B_LOCAL * WORLD)
    sl = slice(rank * B_LOCAL, (rank + 1) * B_LOCAL)
    dyn, keys, err = _run(dyn_all[:, :, sl], keys_all[sl])
    obs = torch.from_numpy(np.ascontiguousarray(dyn.transpose(2, 0, 1)))  # [B_local, nb, 6]
    gathered = torch.empty(WORLD * B_LOCAL, 5, 6)
    dist.all_gather_into_tensor(gathered, obs)
    if rank == 0:
        np.save(out_path, gathered.numpy())
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_rank(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "emu"), "build/libcotix_emu.so"], check=True)
    out = str(tmp_path / "gathered.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(port, out), nprocs=WORLD, join=True)
    gathered = np.load(out)
    dyn_all, keys_all = _initial_state(B_LOCAL * WORLD)
    ref, _, _ = _run(dyn_all, keys_all)
    ref = ref.transpose(2, 0, 1)
    na, nb = np.isnan(gathered), np.isnan(ref)
    assert np.array_equal(na, nb)
    assert np.array_equal(gathered[~na].view(np.uint32), ref[~nb].view(np.uint32))


def test_global_key_slicing_matches_bench():
    """bench.py gives rank r keys split(PRNGKey(3), B*N)[r*B:(r+1)*B]: the
    union over ranks is exactly the single-GPU key set."""
    _setup_paths()
    from cotix_oracle import prng
    full = prng.split(prng.PRNGKey(3), B_LOCAL * WORLD)
    parts = [full[r * B_LOCAL:(r + 1) * B_LOCAL] for r in range(WORLD)]
    assert np.array_equal(np.concatenate(parts), full)
    with pytest.raises(AssertionError):
        assert np.array_equal(parts[0], parts[1])
