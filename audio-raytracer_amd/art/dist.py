"""Fan sharding across ranks (one process per GPU) and the all-gather of per-fan result blocks.

Fans are independent (SURVEY.md §8 e): rank r of W owns fans [S*r//W, S*(r+1)//W). Colliders,
directions and targets are replicated per rank. Each rank's packed fan records (include/
art_device.h art_fan_layout) form one contiguous block; one all_gather_into_tensor over RCCL
(torch.distributed "nccl") — or gloo on CPU — assembles the [S * stride] result on every rank.
Uneven shards are padded to ceil(S/W) records and trimmed after the gather.
"""
from __future__ import annotations


def shard_range(S: int, world: int, rank: int) -> tuple[int, int]:
    return (S * rank) // world, (S * (rank + 1)) // world


def all_gather_fan_blocks(local_block, S: int, stride: int, world: int, group=None):
    """local_block: uint8 tensor [n_local * stride] of this rank's fans (n_local from shard_range).
    Returns a uint8 tensor [S * stride] with every fan's record in global fan order."""
    import torch
    import torch.distributed as dist

    per = (S + world - 1) // world
    n_local = local_block.numel() // stride
    if world == 1:
        return local_block
    if local_block.is_cuda and dist.get_backend(group) == "gloo":  # gloo gathers host buffers
        return all_gather_fan_blocks(local_block.cpu(), S, stride, world, group).to(local_block.device)
    if n_local == per and S == per * world:
        out = torch.empty(S * stride, dtype=torch.uint8, device=local_block.device)
        dist.all_gather_into_tensor(out, local_block, group=group)
        return out
    padded = torch.zeros(per * stride, dtype=torch.uint8, device=local_block.device)
    padded[: n_local * stride] = local_block
    full = torch.empty(world * per * stride, dtype=torch.uint8, device=local_block.device)
    dist.all_gather_into_tensor(full, padded, group=group)
    parts = []
    for r in range(world):
        b, e = shard_range(S, world, r)
        parts.append(full[r * per * stride: (r * per + (e - b)) * stride])
    return torch.cat(parts)


class OverlappedGather:
    """Frames whose all-gather runs beside the next frame's kernels (one process per GPU, RCCL).

    step(): launch(block) writes this frame's result block, then gather(out, block) is issued
    asynchronously (torch.distributed ..., async_op=True: the collective's stream waits for the
    launch stream, the launch stream goes on). Two blocks alternate; before frame i + 2 rewrites
    block i % 2, wait() on gather i makes the launch stream wait for it. drain() waits for every
    pending gather; last() is the output of the most recent one.

    launch(block) enqueues the frame into `block`; gather(out, block) returns a Work-like object
    with wait()."""

    def __init__(self, blocks, outs, launch, gather):
        import collections
        assert len(blocks) == 2 and len(outs) == 2
        self.blocks, self.outs, self.launch, self.gather = blocks, outs, launch, gather
        self.pend = collections.deque()
        self.n = 0

    def step(self):
        i = self.n & 1
        if len(self.pend) == 2:
            self.pend.popleft().wait()  # gather n - 2 read blocks[i]
        self.launch(self.blocks[i])
        self.pend.append(self.gather(self.outs[i], self.blocks[i]))
        self.n += 1

    def drain(self):
        while self.pend:
            self.pend.popleft().wait()

    def last(self):
        return self.outs[(self.n - 1) & 1] if self.n else None
