"""CPU, world_size 2 over gloo: the trajectory exchange step (mzba/shard.py) gathers every
rank's packed records into rank 0 in global env order, and the record packing round-trips."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mzba.shard import TrajectoryGather, pack_records, unpack_records


def _rec(T, B, hw, rank):
    g = torch.Generator().manual_seed(100 + rank)
    return {
        "action": torch.randint(0, 3, (T, B), generator=g, dtype=torch.uint8),
        "mask": torch.randint(0, 2, (T, B), generator=g, dtype=torch.uint8),
        "reward": torch.randn(T, B, generator=g),
        "values": torch.randn(T, B, generator=g),
        "counts": torch.randint(0, 51, (T, B, 3), generator=g, dtype=torch.int64),
        "frame": torch.randint(0, 8, (T, B, hw), generator=g, dtype=torch.uint8),
    }


def test_pack_roundtrip():
    r = _rec(5, 7, 320, 0)
    u = unpack_records(pack_records(r, 1, 4))
    for k in r:
        assert torch.equal(u[k], r[k][1:4]), k


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T, B, hw = 6, 5, 320
    rec = _rec(T, B, hw, rank)
    g = TrajectoryGather(world, rank, 4, B, hw, "cpu", pin=False)
    n = g.exchange(rec, 2, 6)
    if rank == 0:
        got = g.host_records(n)
        out.put({k: v.numpy() for k, v in got.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_gather_world2_global_env_order():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = [_rec(6, 5, 320, r) for r in range(2)]
    for k in ("action", "mask", "reward", "values", "counts", "frame"):
        want = np.concatenate([ref[r][k][2:6].numpy() for r in range(2)], axis=1)
        np.testing.assert_array_equal(got[k], want, err_msg=k)


def test_rng_keyed_on_global_env():
    """Sharding invariance of the keyed stream: rank r's envs draw what the global batch draws."""
    from oracle.env import BreakoutEnvOracle
    from mzba.config import default_config
    cfg = default_config()["environment"]
    full = BreakoutEnvOracle({**cfg, "n_parallel": 16}).reset_params(5, 3)
    for r in range(2):
        part = BreakoutEnvOracle({**cfg, "n_parallel": 8}).reset_params(5, 3, env_offset=8 * r)
        for a, b in zip(part, full):
            np.testing.assert_array_equal(a, b[8 * r: 8 * r + 8])
