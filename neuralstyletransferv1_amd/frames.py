"""Frame sharding across GPUs: round-robin assignment + ordered gather to rank 0.

SURVEY.md §8(e): the forward is per-frame independent (InstanceNorm statistics are per
frame), so frames shard round-robin; the post chain has one ordered dependency (the LAB
EMA state prev_L, pipeline.py:1951-1961), so stylized frames are gathered to rank 0 in frame
order.  With the "nccl" backend (RCCL over xGMI) the gather is point-to-point: each rank
sends its uint8 frames straight to rank 0 over its own link (6.2 MB per 1080p frame).
Host-side pure logic is unit-tested with the gloo backend on CPU tensors.
"""
from __future__ import annotations

from typing import Callable, List, Sequence

import torch
import torch.distributed as dist


def plan_groups(sizes: Sequence[tuple], world: int, batch: int) -> List[List[int]]:
    """Split frame indices 0..len(sizes)-1 into consecutive groups of at most world*batch frames
    that share one frame size (a size change starts a new group, as pipeline.py:1104-1113 resets
    its temporal caches there)."""
    groups: List[List[int]] = []
    cur: List[int] = []
    cap = max(1, world * batch)
    for i, s in enumerate(sizes):
        if cur and (len(cur) == cap or sizes[cur[0]] != s):
            groups.append(cur)
            cur = []
        cur.append(i)
    if cur:
        groups.append(cur)
    return groups


def shard(group: Sequence[int], world: int, rank: int) -> List[int]:
    """Round-robin: the group's j-th frame goes to rank j % world (frame f -> GPU f mod N)."""
    return [f for j, f in enumerate(group) if j % world == rank]


def gather_ordered(local: torch.Tensor, group: Sequence[int], world: int, rank: int, dst: int = 0):
    """Collect each rank's shard (frames in shard() order, stacked on dim 0) on `dst`, returned
    in group order; other ranks return None.  Point-to-point sends (no collective on the rest)."""
    if world == 1:
        return local
    n = len(group)
    if rank != dst:
        if local.shape[0] > 0:
            dist.send(local.contiguous(), dst)
        return None
    out = torch.empty((n,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = [j for j in range(n) if j % world == r]
        if not idx:
            continue
        if r == dst:
            buf = local
        else:
            buf = torch.empty((len(idx),) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
            dist.recv(buf, r)
        out[idx] = buf
    return out


def run_sharded(groups: Sequence[Sequence[int]], world: int, rank: int,
                stylize: Callable[[List[int]], torch.Tensor], consume: Callable[[List[int], torch.Tensor], None]):
    """Drive the loop: every rank stylizes its shard of each group; `dst` consumes in order."""
    for g in groups:
        mine = shard(g, world, rank)
        local = stylize(mine)
        full = gather_ordered(local, g, world, rank)
        if full is not None:
            consume(list(g), full)
