"""CPU, world_size 2 over gloo: the two collectives of mzba/shard.py as bench.py runs them for
N > 1 — the target-net refresh (rank 0's state_dict broadcast to every rank, train_torch.py:137-139)
and the trajectory sink (every rank's packed records gathered to rank 0 in global env order) — and
the record packing round trip."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mzba.shard import TrajectoryGather, broadcast_state_dict, pack_records, unpack_records


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


def _mcfg():
    from mzba.config import default_config, small_model_cfg
    return small_model_cfg(default_config())


def test_pack_roundtrip():
    r = _rec(5, 7, 320, 0)
    u = unpack_records(pack_records(r, 1, 4))
    for k in r:
        assert torch.equal(u[k], r[k][1:4]), k


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mzba.weights import init_state_dict
    # target-net refresh: only rank 0 holds the learner's weights
    sd = init_state_dict(_mcfg(), 3) if rank == 0 else None
    if rank == 0:
        sd["dyn_net.conv_block.bn.num_batches_tracked"] = np.array(17, np.int64)
    got_sd = broadcast_state_dict(_mcfg(), sd, "cpu")
    T, B, hw = 6, 5, 320
    rec = _rec(T, B, hw, rank)
    g = TrajectoryGather(world, rank, 4, B, hw, "cpu", pin=False)
    n = g.exchange(rec, 2, 6)
    res = {"sd": {k: v.numpy() for k, v in got_sd.items()}}
    if rank == 0:
        assert g.gathered is not None and g.host is not None
        res["rec"] = {k: v.numpy() for k, v in g.host_records(n).items()}
    else:
        assert g.gathered is None and g.host is None  # gather to the root: nothing lands here
    out.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_and_gather_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(2))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    from mzba.weights import init_state_dict
    want_sd = init_state_dict(_mcfg(), 3)
    want_sd["dyn_net.conv_block.bn.num_batches_tracked"] = np.array(17, np.int64)
    for r in range(2):
        assert list(got[r]["sd"]) == list(want_sd)
        for k, v in want_sd.items():
            np.testing.assert_array_equal(got[r]["sd"][k], v, err_msg=f"rank {r} {k}")
    ref = [_rec(6, 5, 320, r) for r in range(2)]
    for k in ("action", "mask", "reward", "values", "counts", "frame"):
        want = np.concatenate([ref[r][k][2:6].numpy() for r in range(2)], axis=1)
        np.testing.assert_array_equal(got[0]["rec"][k], want, err_msg=k)


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


def test_sharded_sampling_oracle_equals_global():
    """The temperature step on a shard (its env_offset in the global (n, 3) batch tensor) equals the
    global step's rows: which torch pow lane an element takes depends on its global position."""
    from oracle.acting import sample_probs
    c = np.random.default_rng(0).integers(0, 51, (1029, 3))
    full = sample_probs(c, 0.7)
    for off, n in ((0, 515), (515, 514)):
        np.testing.assert_array_equal(sample_probs(c[off:off + n], 0.7, env_offset=off, n_envs_total=1029)
                                      .view(np.uint32), full[off:off + n].view(np.uint32))


def _sink_worker(rank, world, port, out):
    """One rank of a sharded episode through mzba.shard.ShardedSink: its records are written row by row
    (as ActingLoop.act does), pushed every k = 4 rows, and the ranks stop together when every env of
    every rank is done (all_ranks_done). Rank 0 returns the global records."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mzba.shard import ShardedSink, all_ranks_done
    B, hw, Tmax = 5, 320, 20
    rec = _rec(Tmax, B, hw, rank)
    done_at = [6, 11][rank]  # rank 0's envs finish first: it keeps stepping until rank 1's do too
    frame0 = torch.randint(0, 8, (B * hw,), generator=torch.Generator().manual_seed(7 + rank), dtype=torch.uint8)
    sink = ShardedSink(world, rank, 4, B, hw, Tmax, "cpu")
    sink.begin(frame0)
    t = 0
    while not all_ranks_done(torch.full((B,), int(t >= done_at), dtype=torch.uint8)) and t < Tmax:
        t += 1  # the loop wrote row t - 1
        sink.push(rec, t)
    g, f0 = sink.finish(rec, t)
    res = {"t": t}
    if rank == 0:
        res["rec"] = {k: v[:t].numpy() for k, v in g.items()}
        res["frame0"] = f0.numpy()
    else:
        assert g is None and f0 is None
    out.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_sink_assembles_the_global_episode_world2():
    """ActingStage's N > 1 sink on CPU collectives: two ranks' record rows, gathered every 4 steps,
    land in rank 0's (T, 2B, ...) episode tensors in global env order, the frames g(s0) of both
    ranks with them; the ranks stop on the same step (the global batch's all-done)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sink_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(2))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0]["t"] == got[1]["t"] == 11
    ref = [_rec(20, 5, 320, r) for r in range(2)]
    for k in ("action", "mask", "reward", "values", "counts", "frame"):
        want = np.concatenate([ref[r][k][:11].numpy() for r in range(2)], axis=1)
        np.testing.assert_array_equal(got[0]["rec"][k], want, err_msg=k)
    f0 = [torch.randint(0, 8, (5 * 320,), generator=torch.Generator().manual_seed(7 + r), dtype=torch.uint8)
          for r in range(2)]
    np.testing.assert_array_equal(got[0]["frame0"], torch.cat(f0).view(10, 320).numpy())


def test_exchange_refuses_world_gt1_without_process_group():
    g = TrajectoryGather(2, 0, 4, 3, 320, "cpu", pin=False)
    with pytest.raises(RuntimeError):
        g.exchange(_rec(4, 3, 320, 0), 0, 4)
