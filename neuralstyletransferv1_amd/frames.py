"""Frame sharding across GPUs: round-robin assignment + ordered gather to rank 0.

SURVEY.md §8(e): the forward is per-frame independent (InstanceNorm statistics are per
frame), so frames shard round-robin; the post chain has one ordered dependency (the LAB
EMA state prev_L, pipeline.py:1951-1961), so stylized frames are gathered to rank 0 in frame
order.  With the "nccl" backend (RCCL over xGMI) the gather is point-to-point: each rank
sends its uint8 frames straight to rank 0 over its own link (6.2 MB per 1080p frame).
Host-side pure logic is unit-tested with the gloo backend on CPU tensors.  With the gloo backend
(tests; several ranks sharing one GPU) device tensors travel through host memory.

The exchange of a group is posted as one batch of point-to-point ops (rank 0 receives from every peer at
once) and completed one group later, so it overlaps the next group's forward; rank 0, which also runs the
ordered post chain, stylizes a lighter share of each group (rank0_share).

Failure handling: before each group's exchange every rank contributes a status flag to one tiny
all-reduce (the stylize of this group and the consume of the previous one), so a rank that fails
makes every rank raise instead of leaving the others blocked in send/recv.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist


# Rank 0 also runs the ordered post chain of every rank's frames (LAB EMA, blend: ~0.021 ms per 1080p frame
# against ~0.64 ms per frame of forward), so it takes a lighter share of each group:
# batch - round(world * batch * EMA_COST_RATIO) frames (8 GPUs, batch 8: 6 frames; everyone else 8).
EMA_COST_RATIO = 0.033


def rank0_share(world: int, batch: int) -> int:
    """Frames rank 0 stylizes per group (the others stylize `batch`)."""
    if world <= 1:
        return batch
    return max(1, batch - int(round(world * batch * EMA_COST_RATIO)))


def _caps(world: int, batch: int, rank0_batch=None) -> List[int]:
    return [batch if rank0_batch is None else rank0_batch] + [batch] * (world - 1)


def plan_groups(sizes: Sequence[tuple], world: int, batch: int, rank0_batch=None) -> List[List[int]]:
    """Split frame indices 0..len(sizes)-1 into consecutive groups of at most sum(caps) frames (every rank's
    share: `batch`, rank 0 `rank0_batch` when given) that share one frame size (a size change starts a new
    group, as pipeline.py:1104-1113 resets its temporal caches there)."""
    groups: List[List[int]] = []
    cur: List[int] = []
    cap = max(1, sum(_caps(world, batch, rank0_batch)))
    for i, s in enumerate(sizes):
        if cur and (len(cur) == cap or sizes[cur[0]] != s):
            groups.append(cur)
            cur = []
        cur.append(i)
    if cur:
        groups.append(cur)
    return groups


def owners(n: int, world: int, caps: Optional[Sequence[int]] = None) -> List[int]:
    """Rank of each of a group's n frames: round-robin (frame j -> rank j % world) over the ranks that still
    have room for this group (caps[r] frames; no caps = unbounded)."""
    if caps is None:
        return [j % world for j in range(n)]
    left = list(caps)
    out, r = [], 0
    for _ in range(n):
        for _k in range(world):
            if left[r] > 0:
                break
            r = (r + 1) % world
        else:
            raise ValueError("group larger than the ranks' shares")
        out.append(r)
        left[r] -= 1
        r = (r + 1) % world
    return out


def shard(group: Sequence[int], world: int, rank: int, caps: Optional[Sequence[int]] = None) -> List[int]:
    """This rank's frames of a group, in group order (owners())."""
    own = owners(len(group), world, caps)
    return [f for f, o in zip(group, own) if o == rank]


def _via_host() -> bool:
    return dist.is_initialized() and dist.get_backend() == "gloo"


class Exchange:
    """An ordered gather in flight: the point-to-point sends of this rank, or (on dst) the receives of every
    peer, posted together (batch_isend_irecv: one RCCL group, every xGMI link at once) and completed by
    gather_finish, so the transfer runs while the caller stylizes the next group."""

    def __init__(self, works, result=None, parts=None, n=0, owner=None, keep=None, device=None, shape=None,
                 dtype=None):
        self.works, self.result, self.parts, self.n, self.owner = works, result, parts, n, owner
        self.keep, self.device, self.shape, self.dtype = keep, device, shape, dtype


def gather_start(local: torch.Tensor, group: Sequence[int], world: int, rank: int,
                 caps: Optional[Sequence[int]] = None, dst: int = 0) -> Exchange:
    """Post the exchange of one group: each rank's shard (frames in shard() order, stacked on dim 0) to dst."""
    if world == 1:
        return Exchange([], result=local)
    n = len(group)
    own = owners(n, world, caps)
    host = _via_host() and local.device.type != "cpu"
    if rank != dst:
        if local.shape[0] == 0:
            return Exchange([])
        t = local.contiguous().cpu() if host else local.contiguous()
        return Exchange(dist.batch_isend_irecv([dist.P2POp(dist.isend, t, dst)]), keep=t)
    parts, ops = {}, []
    for r in range(world):
        k = sum(1 for o in own if o == r)
        if k == 0 or r == dst:
            continue
        buf = torch.empty((k,) + tuple(local.shape[1:]), dtype=local.dtype, device="cpu" if host else local.device)
        parts[r] = buf
        ops.append(dist.P2POp(dist.irecv, buf, r))
    parts[dst] = local
    works = dist.batch_isend_irecv(ops) if ops else []
    return Exchange(works, parts=parts, n=n, owner=own, device=local.device, shape=tuple(local.shape[1:]),
                    dtype=local.dtype)


def gather_finish(ex: Exchange):
    """Wait for an exchange; on dst the group's frames in group order, elsewhere None."""
    for w in ex.works or []:
        w.wait()
    if ex.result is not None or ex.parts is None:
        return ex.result
    out = torch.empty((ex.n,) + ex.shape, dtype=ex.dtype, device=ex.device)
    for r, buf in ex.parts.items():
        idx = [j for j, o in enumerate(ex.owner) if o == r]
        if idx:
            out[idx] = buf.to(ex.device)
    return out


def gather_ordered(local: torch.Tensor, group: Sequence[int], world: int, rank: int, dst: int = 0,
                   caps: Optional[Sequence[int]] = None):
    """Blocking form: collect each rank's shard on `dst` in group order; other ranks return None."""
    return gather_finish(gather_start(local, group, world, rank, caps, dst))


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
                device: torch.device = torch.device("cpu"), caps: Optional[Sequence[int]] = None):
    """Drive the loop: every rank stylizes its shard of each group; `dst` consumes in order.  Double-buffered:
    group k's exchange is posted after every rank has agreed group k stylized fine, and completed (and
    consumed on dst) after group k+1's stylize has been issued, so the transfer overlaps that forward.  A
    failure on any rank (its stylize, or rank 0's consume of the previous group) reaches every rank through
    agree_ok before the next exchange: the failing rank re-raises its own error, the others raise RankFailed;
    the group before the failure is still consumed."""
    s_err = c_err = None
    pend = None

    def drain():
        nonlocal pend, c_err
        if pend is None:
            return
        pg, ex = pend
        pend = None
        full = gather_finish(ex)
        if full is not None and c_err is None:
            try:
                consume(list(pg), full)
            except Exception as e:  # noqa: BLE001 -- re-raised below on this rank
                if world == 1:
                    raise
                c_err = e
    for g in groups:
        mine = shard(g, world, rank, caps)
        local = None
        if s_err is None:
            try:
                local = stylize(mine)
            except Exception as e:  # noqa: BLE001 -- re-raised below on this rank
                s_err = e
        drain()  # the previous group's exchange ran beside this stylize
        err = s_err or c_err
        if world > 1:
            agree_ok(err is None, device)
        if err is not None:
            raise err
        pend = (g, gather_start(local, g, world, rank, caps))
    drain()
    err = s_err or c_err
    if world > 1:
        agree_ok(err is None, device)
    if err is not None:
        raise err
