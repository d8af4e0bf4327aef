"""Frame sharding across GPUs: round-robin assignment + ordered gather to rank 0.

SURVEY.md §8(e): the forward is per-frame independent (InstanceNorm statistics are per
frame), so frames shard round-robin; the post chain has one ordered dependency (the LAB
EMA state prev_L, pipeline.py:1951-1961), so stylized frames are gathered to rank 0 in frame
order.  With the "nccl" backend (RCCL over xGMI) the gather is point-to-point: each rank
sends its uint8 frames straight to rank 0 over its own link (6.2 MB per 1080p frame).
Host-side pure logic is unit-tested with the gloo backend on CPU tensors.  With the gloo backend
(tests; several ranks sharing one GPU) device tensors travel through host memory.

Failure handling: before each group's exchange every rank contributes a status flag to one tiny
all-reduce (the stylize of this group and the consume of the previous one), so a rank that fails
makes every rank raise instead of leaving the others blocked in send/recv.
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


def _via_host() -> bool:
    return dist.is_initialized() and dist.get_backend() == "gloo"


def gather_ordered(local: torch.Tensor, group: Sequence[int], world: int, rank: int, dst: int = 0):
    """Collect each rank's shard (frames in shard() order, stacked on dim 0) on `dst`, returned
    in group order; other ranks return None.  Point-to-point sends (no collective on the rest)."""
    if world == 1:
        return local
    n = len(group)
    host = _via_host() and local.device.type != "cpu"
    if rank != dst:
        if local.shape[0] > 0:
            dist.send(local.contiguous().cpu() if host else local.contiguous(), dst)
        return None
    out = torch.empty((n,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = [j for j in range(n) if j % world == r]
        if not idx:
            continue
        if r == dst:
            buf = local
        else:
            buf = torch.empty((len(idx),) + tuple(local.shape[1:]), dtype=local.dtype,
                              device="cpu" if host else local.device)
            dist.recv(buf, r)
            buf = buf.to(local.device)
        out[idx] = buf
    return out


class RankFailed(RuntimeError):
    """Another rank of the job failed; this rank stops instead of blocking in the exchange."""


def agree_ok(ok: bool, device: torch.device) -> None:
    """All ranks learn whether every rank is fine (MAX all-reduce of a failure flag)."""
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32,
                        device="cpu" if _via_host() else device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()) and ok:
        raise RankFailed("another rank failed; stopping this one")


def run_sharded(groups: Sequence[Sequence[int]], world: int, rank: int,
                stylize: Callable[[List[int]], torch.Tensor], consume: Callable[[List[int], torch.Tensor], None],
                device: torch.device = torch.device("cpu")):
    """Drive the loop: every rank stylizes its shard of each group; `dst` consumes in order.
    A failure on any rank (its stylize, or rank 0's consume of the previous group) reaches every
    rank through agree_ok before the next exchange: the failing rank re-raises its own error, the
    others raise RankFailed."""
    err = None
    for g in groups:
        mine = shard(g, world, rank)
        local = None
        if err is None:
            try:
                local = stylize(mine)
            except Exception as e:  # noqa: BLE001 -- re-raised below on this rank
                err = e
        if world > 1:
            try:
                agree_ok(err is None, device)
            except RankFailed:
                raise
            if err is not None:
                raise err
        elif err is not None:
            raise err
        full = gather_ordered(local, g, world, rank)
        if full is not None:
            try:
                consume(list(g), full)
            except Exception as e:  # noqa: BLE001
                if world == 1:
                    raise
                err = e
    if world > 1:
        agree_ok(err is None, device)
    if err is not None:
        raise err
