"""Env sharding across ranks: the trajectory sink (records -> rank 0) and the target-net
refresh (rank 0's weights -> every rank).

Envs are independent during acting (BN in eval mode, per-env min-max scaling, no
cross-env term in step or search — SURVEY §8(e)), so rank r simply owns global envs
[r*B, (r+1)*B) and every random draw is keyed by the GLOBAL env id: results are
identical for any world size. Two collectives, both where the reference has a real
exchange:
  * the sink — each rank's per-step ObservationTrajectory rows (replay_buffer.py:17-35)
    are packed into one byte slab per k steps and GATHERED to rank 0 (RCCL over xGMI
    with backend "nccl"; gloo in the CPU tests): only rank 0 consumes records (its host
    replay buffer), so a gather moves 1/N of an all-gather's bytes; rank 0 copies them
    to pinned host memory behind an event;
  * the target-net refresh (train_torch.py:137-139, load_latest_weights :361-367) — rank 0
    holds the learner's state_dict, one flat f32 broadcast (+ one int64 broadcast for the
    BN batch counters) hands it to every acting rank, which re-packs its agent.

Record layout per (step, env), little-endian, REC_BYTES = 28 + HW:
  action u8 | mask u8 | pad u16 | reward f32 | value f32 | counts i32[3] | pad u32 | frame u8[HW]
"""
import contextlib
from collections import OrderedDict

import numpy as np
import torch
import torch.distributed as dist

from .weights import state_dict_spec

HDR = 28


def rec_bytes(hw):
    return HDR + hw


def pack_records(rec, t0, t1, out=None):
    """rec: dict of (T,B,...) tensors (acting-loop sink). Returns (t1-t0, B, REC_BYTES) u8."""
    a, m = rec["action"][t0:t1], rec["mask"][t0:t1]
    T, B = a.shape
    fr = rec.get("frame")
    hw = fr.shape[-1] if fr is not None else 0
    if out is None:
        out = torch.zeros(T, B, rec_bytes(hw), dtype=torch.uint8, device=a.device)
    out[:, :, 0] = a
    out[:, :, 1] = m
    out[:, :, 4:8] = rec["reward"][t0:t1].contiguous().view(torch.uint8).view(T, B, 4)
    out[:, :, 8:12] = rec["values"][t0:t1].contiguous().view(torch.uint8).view(T, B, 4)
    out[:, :, 12:24] = rec["counts"][t0:t1].to(torch.int32).contiguous().view(torch.uint8).view(T, B, 12)
    if hw:
        out[:, :, HDR:] = fr[t0:t1]
    return out


def unpack_records(buf):
    """(..., REC_BYTES) u8 -> dict of tensors (inverse of pack_records)."""
    sh = buf.shape[:-1]
    b = buf.contiguous()
    return {
        "action": b[..., 0].clone(),
        "mask": b[..., 1].clone(),
        "reward": b[..., 4:8].contiguous().view(torch.float32).view(sh),
        "values": b[..., 8:12].contiguous().view(torch.float32).view(sh),
        "counts": b[..., 12:24].contiguous().view(torch.int32).view(*sh, 3).to(torch.int64),
        "frame": b[..., HDR:].clone(),
    }


class TrajectoryGather:
    """Gather of packed record slabs to rank 0, then into its pinned host buffer.

    On a GPU the whole exchange (pack, RCCL gather, D2H copy) runs on a side stream behind an event
    recorded on the acting stream, so it overlaps the next acting steps; `fence()` makes the acting
    stream wait for the last pack before record rows are reused (a new episode restarts at row 0)."""

    def __init__(self, world_size, rank, k_steps, B, hw, device, pin=True):
        self.ws, self.rank, self.k, self.B, self.hw = world_size, rank, k_steps, B, hw
        self.device = torch.device(device)
        self.slab = torch.zeros(k_steps, B, rec_bytes(hw), dtype=torch.uint8, device=self.device)
        self.gathered = self.host = self.copied = None
        self.side = self.packed = None
        if rank == 0:
            self.gathered = torch.zeros(world_size, k_steps, B, rec_bytes(hw), dtype=torch.uint8, device=self.device)
            self.host = torch.zeros(world_size, k_steps, B, rec_bytes(hw), dtype=torch.uint8,
                                    pin_memory=pin and self.device.type == "cuda")

    def exchange(self, rec, t0, t1, into=None, to_host=True):
        """Records of steps [t0, t1) (t1 - t0 <= k) of every rank -> rank 0. Every rank calls it.
        With torch.distributed initialised the collective runs at any world size (RCCL on the
        device with backend "nccl"; gloo moves host copies). Rank 0 then unpacks the rows into
        `into` (a dict of (T, world*B, ...) device tensors in global env order, rows [t0, t1)) and/or
        copies them to its pinned host buffer (`to_host`), on the same side stream."""
        n = t1 - t0
        if not 0 < n <= self.k:
            raise ValueError(f"exchange: {n} rows, the slab holds 1..{self.k}")
        distributed = dist.is_available() and dist.is_initialized()
        if self.ws > 1 and not distributed:
            raise RuntimeError("TrajectoryGather: world_size > 1 needs torch.distributed initialised")
        cuda = self.device.type == "cuda"
        if cuda:
            if self.side is None:
                self.side = torch.cuda.Stream(device=self.device)
            ready = torch.cuda.Event()
            ready.record()  # every record row written so far (acting stream)
            self.side.wait_event(ready)
            stream = torch.cuda.stream(self.side)
        else:
            stream = contextlib.nullcontext()
        with stream:
            pack_records(rec, t0, t1, self.slab[:n])
            if cuda:
                self.packed = torch.cuda.Event()
                self.packed.record()
            if distributed:
                if dist.get_backend() == "gloo" and cuda:
                    # gloo gathers host tensors only (CPU tests, and bench.py's one-GPU rehearsal)
                    gl = [torch.empty_like(self.slab, device="cpu") for _ in range(self.ws)] if self.rank == 0 else None
                    dist.gather(self.slab.cpu(), gl, dst=0)
                    if self.rank == 0:
                        self.gathered.copy_(torch.stack(gl))
                else:
                    gl = list(self.gathered.unbind(0)) if self.rank == 0 else None
                    dist.gather(self.slab, gl, dst=0)
            elif self.rank == 0:
                self.gathered[0].copy_(self.slab)
            if self.rank == 0 and into is not None:
                g = self.gathered[:, :n].permute(1, 0, 2, 3).reshape(n, self.ws * self.B, -1)
                for k, v in unpack_records(g).items():
                    if into.get(k) is not None:
                        into[k][t0:t1].copy_(v)
            if self.rank == 0 and to_host:
                self.host.copy_(self.gathered, non_blocking=True)
                if cuda:  # host_records() waits for exactly this copy
                    self.copied = torch.cuda.Event()
                    self.copied.record()
            if cuda:
                self.landed = torch.cuda.Event()
                self.landed.record()
        return n

    def wait_landed(self):
        """The current stream waits for the last exchange's unpack into `into` (rank 0)."""
        if getattr(self, "landed", None) is not None:
            torch.cuda.current_stream(self.device).wait_event(self.landed)

    def fence(self):
        """The acting stream waits until the last exchange has packed its rows (call before the
        record rows are overwritten, e.g. before ActingLoop.reset)."""
        if self.packed is not None:
            torch.cuda.current_stream(self.device).wait_event(self.packed)

    def host_records(self, n):
        """rank 0: dict of (n, world*B, ...) in global env order."""
        if self.copied is not None:
            self.copied.synchronize()
        h = self.host[:, :n].permute(1, 0, 2, 3).reshape(n, self.ws * self.B, -1)
        return unpack_records(h)


def gather_rows(x, world_size, rank):
    """Rank 0 <- every rank's (B, ...) tensor, concatenated in rank order (global env order); the other
    ranks get None. Used once per episode for the g(s0) frames the padded trajectories start from
    (train_torch.py:167, _pad_initial_state :313-332)."""
    if world_size == 1:
        return x
    gloo_cuda = dist.get_backend() == "gloo" and x.device.type == "cuda"
    src = x.cpu() if gloo_cuda else x.contiguous()
    gl = [torch.empty_like(src) for _ in range(world_size)] if rank == 0 else None
    dist.gather(src, gl, dst=0)
    return torch.cat(gl).to(x.device) if rank == 0 else None


def all_ranks_done(local_done):
    """True when every env of every rank is done (`torch.all(done_mask == True)` over the global batch,
    train_torch.py:184): the ranks keep stepping in lockstep until then, so the step index, the search
    id and every keyed draw stay those of the one global loop. local_done: this rank's done flags."""
    live = (local_done != 0).logical_not().any().to(torch.int32).reshape(1)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo" and live.device.type == "cuda":
            live = live.cpu()
        dist.all_reduce(live, op=dist.ReduceOp.MAX)
    return int(live.item()) == 0


class ShardedSink:
    """Rank 0's device copy of one episode's records of ALL ranks, in global env order: every k steps the
    ranks' record rows go through a TrajectoryGather straight into (T, world*B, ...) tensors, which the
    replay ingest (replay_buffer.py:96-165 via DeviceReplayBuffer.ingest_records) and the trajectory
    lists read as if one loop had run the global batch. Every rank calls begin / push / finish."""

    KEYS = ("action", "reward", "mask", "frame", "counts", "values")

    def __init__(self, world_size, rank, k_steps, B, hw, max_steps, device):
        self.ws, self.rank, self.k, self.B, self.hw = world_size, rank, k_steps, B, hw
        self.device = torch.device(device)
        self.gather = TrajectoryGather(world_size, rank, k_steps, B, hw, device, pin=False)
        self.rec = self.frame0 = None
        if rank == 0:
            n, T, dev = world_size * B, max_steps, self.device
            self.rec = {"action": torch.zeros(T, n, dtype=torch.uint8, device=dev),
                        "reward": torch.zeros(T, n, dtype=torch.float32, device=dev),
                        "mask": torch.zeros(T, n, dtype=torch.uint8, device=dev),
                        "frame": torch.zeros(T, n, hw, dtype=torch.uint8, device=dev),
                        "counts": torch.zeros(T, n, 3, dtype=torch.int64, device=dev),
                        "values": torch.zeros(T, n, dtype=torch.float32, device=dev)}
        self.t0 = 0

    def begin(self, frame0):
        """A new episode: frame0 = this rank's u8 g(s0) codes (B, H*W)."""
        self.gather.fence()  # the loop's record rows restart at 0: after the last pack read them
        self.frame0 = gather_rows(frame0.reshape(self.B, self.hw), self.ws, self.rank)
        self.t0 = 0

    def push(self, rec, t, final=False):
        """The loop has written rows [0, t): exchange the rows since the last push every k steps (and
        at the end of the episode)."""
        if t - self.t0 >= self.k or (final and t > self.t0):
            while self.t0 < t:
                t1 = min(t, self.t0 + self.k)
                self.gather.exchange(rec, self.t0, t1, into=self.rec, to_host=False)
                self.t0 = t1

    def finish(self, rec, t):
        """End of episode (t rows): rank 0 gets (records, frame0) in global env order, ready on its
        current stream; the other ranks get (None, None)."""
        self.push(rec, t, final=True)
        if self.device.type == "cuda":
            self.gather.wait_landed()
        return (self.rec, self.frame0) if self.rank == 0 else (None, None)


def broadcast_state_dict(mcfg, state_dict, device, src=0):
    """Target-net refresh across ranks (train_torch.py:137-139, :361-367): `src` passes the learner's
    reference-format state_dict (tensors or arrays), the other ranks pass None; every rank returns
    the same OrderedDict of CPU tensors in networks.py key order. Two collectives: the float
    entries flattened into one f32 buffer, the BN `num_batches_tracked` counters into one int64."""
    rank = dist.get_rank()
    spec = state_dict_spec(mcfg)
    fkeys = [(k, s) for k, s in spec if not k.endswith("num_batches_tracked")]
    ikeys = [k for k, _ in spec if k.endswith("num_batches_tracked")]
    nf = sum(int(np.prod(s)) for _, s in fkeys)
    dev = torch.device(device)
    fbuf = torch.empty(nf, dtype=torch.float32, device=dev)
    ibuf = torch.zeros(max(len(ikeys), 1), dtype=torch.int64, device=dev)
    if rank == src:
        if state_dict is None:
            raise ValueError("broadcast_state_dict: the source rank must pass the state_dict")
        fbuf.copy_(torch.cat([torch.as_tensor(np.asarray(state_dict[k]), dtype=torch.float32).reshape(-1)
                              for k, _ in fkeys]))
        if ikeys:
            ibuf.copy_(torch.tensor([int(np.asarray(state_dict[k])) for k in ikeys], dtype=torch.int64))
    dist.broadcast(fbuf, src)
    dist.broadcast(ibuf, src)
    fh, ih = fbuf.cpu(), ibuf.cpu()
    out, o = OrderedDict(), 0
    for k, s in spec:
        if k.endswith("num_batches_tracked"):
            out[k] = ih[ikeys.index(k)].clone()
        else:
            n = int(np.prod(s))
            out[k] = fh[o:o + n].view(s).clone()
            o += n
    return out


def refresh_target(agent, mcfg, state_dict, device, src=0):
    """The acting ranks' target net <- rank src's learner weights (load_latest_weights). The agent
    copies them into its packed device buffers in place (MuZeroAgent.load_state_dict), so acting
    loops already built on it — and their captured step graphs — run the new weights next step."""
    sd = broadcast_state_dict(mcfg, state_dict, device, src)
    agent.load_state_dict({k: v.numpy() for k, v in sd.items()})
    return sd
