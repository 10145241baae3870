"""Env sharding across ranks + the one exchange step: trajectory records -> rank 0.

Envs are independent during acting (BN in eval mode, per-env min-max scaling, no
cross-env term in step or search — SURVEY §8(e)), so rank r simply owns global envs
[r*B, (r+1)*B) and every random draw is keyed by the GLOBAL env id: results are
identical for any world size. The only collective is the reference's sink: each
rank's per-step ObservationTrajectory rows (replay_buffer.py:17-35) are packed into
one byte slab per k steps and all-gathered (RCCL over xGMI with backend "nccl"; gloo
in the CPU tests) into rank 0, which copies them to pinned host memory.

Record layout per (step, env), little-endian, REC_BYTES = 28 + HW:
  action u8 | mask u8 | pad u16 | reward f32 | value f32 | counts i32[3] | pad u32 | frame u8[HW]
"""
import torch
import torch.distributed as dist

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
    """All-gather of packed record slabs into rank 0's host buffer (pinned)."""

    def __init__(self, world_size, rank, k_steps, B, hw, device, pin=True):
        self.ws, self.rank, self.k, self.B, self.hw = world_size, rank, k_steps, B, hw
        self.device = torch.device(device)
        self.slab = torch.zeros(k_steps, B, rec_bytes(hw), dtype=torch.uint8, device=self.device)
        self.gathered = torch.zeros(world_size, k_steps, B, rec_bytes(hw), dtype=torch.uint8, device=self.device)
        self.host = None
        if rank == 0:
            self.host = torch.zeros(world_size, k_steps, B, rec_bytes(hw), dtype=torch.uint8,
                                    pin_memory=pin and self.device.type == "cuda")

    def exchange(self, rec, t0, t1):
        n = t1 - t0
        pack_records(rec, t0, t1, self.slab[:n])
        if self.ws > 1:
            if dist.get_backend() == "nccl":  # RCCL over xGMI: one flat all-gather
                dist.all_gather_into_tensor(self.gathered.view(-1), self.slab.view(-1))
            else:  # gloo (CPU tests)
                dist.all_gather(list(self.gathered.unbind(0)), self.slab)
        else:
            self.gathered[0].copy_(self.slab)
        if self.rank == 0:
            self.host.copy_(self.gathered, non_blocking=True)
        return n

    def host_records(self, n):
        """rank 0: dict of (n, world*B, ...) in global env order."""
        h = self.host[:, :n].permute(1, 0, 2, 3).reshape(n, self.ws * self.B, -1)
        return unpack_records(h)
