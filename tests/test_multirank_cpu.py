"""Multi-GPU path on CPU: world_size-2 gloo.  Each rank owns a contiguous env
range (global ids rank*B .. rank*B+B-1) and BUILDS it itself from those ids
(collider keys and ball perturbations from ONE global split, only global env
0 unperturbed -- the sharded constructor bench.py uses), steps it with the fused kernel's logic (host
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
    """RoboCup reset state for B envs (ball perturbed per env) + global keys,
    built by the golden generator (independent of the sharded constructor)."""
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


def _shard_state(rank):
    """This rank's shard from its global env ids only (cport.robocup_batch with
    offset/total: the oracle side of RoboCupEnv(env_offset, total_envs))."""
    _setup_paths()
    from cotix_oracle import cport
    return cport.robocup_batch(B_LOCAL, offset=rank * B_LOCAL, total=B_LOCAL * WORLD)


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
    dyn, keys, err = _run(*_shard_state(rank))
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


def test_sharded_constructor_matches_global_batch():
    """Each rank's self-built shard is exactly its slice of the global batch:
    rank 1's envs are perturbed (not copies of rank 0's), and only global env
    0 holds the reference state."""
    dyn_all, keys_all = _initial_state(B_LOCAL * WORLD)
    for r in range(WORLD):
        d, k = _shard_state(r)
        sl = slice(r * B_LOCAL, (r + 1) * B_LOCAL)
        assert np.array_equal(d.view(np.uint32), dyn_all[:, :, sl].view(np.uint32))
        assert np.array_equal(k, keys_all[sl])
    d1, _ = _shard_state(1)
    d0, _ = _shard_state(0)
    assert not np.array_equal(d0[4], d1[4])


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
