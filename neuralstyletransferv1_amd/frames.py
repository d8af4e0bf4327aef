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
                 dtype=None, ops=None):
        self.works, self.result, self.parts, self.n, self.owner = works, result, parts, n, owner
        self.keep, self.device, self.shape, self.dtype = keep, device, shape, dtype
        self.ops = ops or []


def gather_start(local: torch.Tensor, group: Sequence[int], world: int, rank: int,
                 caps: Optional[Sequence[int]] = None, dst: int = 0, post: bool = True) -> Exchange:
    """Post the exchange of one group: each rank's shard (frames in shard() order, stacked on dim 0) to dst.  With
    post=False the point-to-point ops are left in `.ops` for the caller to post in a larger batch (run_pipeline)."""
    if world == 1:
        return Exchange([], result=local)
    n = len(group)
    own = owners(n, world, caps)
    if rank != dst and (local is None or local.shape[0] == 0):
        return Exchange([])
    host = _via_host() and local.device.type != "cpu"
    if rank != dst:
        t = local.contiguous().cpu() if host else local.contiguous()
        ops = [dist.P2POp(dist.isend, t, dst)]
        return Exchange(_post(ops) if post else [], keep=t, ops=ops)
    parts, ops = {}, []
    for r in range(world):
        k = sum(1 for o in own if o == r)
        if k == 0 or r == dst:
            continue
        buf = torch.empty((k,) + tuple(local.shape[1:]), dtype=local.dtype, device="cpu" if host else local.device)
        parts[r] = buf
        ops.append(dist.P2POp(dist.irecv, buf, r))
    parts[dst] = local
    return Exchange(_post(ops) if post else [], parts=parts, n=n, owner=own, device=local.device,
                    shape=tuple(local.shape[1:]), dtype=local.dtype, ops=ops)


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


class _Return:
    """The return leg of a group in flight: dst's rows for each owner (point-to-point sends), or an owner's receive
    buffer.  `result` = this rank's rows (its frames of the group, in shard order) once the leg has completed."""

    def __init__(self, ops, result=None, buf=None, device=None, keep=None):
        self.ops, self.result, self.buf, self.device, self.keep = ops, result, buf, device, keep
        self.works = []

    def finish(self):
        for w in self.works:
            w.wait()
        if self.buf is not None:
            return self.buf.to(self.device) if self.buf.device != self.device else self.buf
        return self.result


def return_ops(rows: Optional[torch.Tensor], group: Sequence[int], world: int, rank: int, spec,
               caps: Optional[Sequence[int]] = None, src: int = 0, device: torch.device = torch.device("cpu")) -> _Return:
    """The return leg of one group (posted together with the next group's gather, run_pipeline): on src, `rows`
    holds the group's per-frame results in group order and each owner's rows are sent back to it; every other
    rank receives its own rows (shard order) into a buffer of `spec` = (per-frame shape, dtype)."""
    own = owners(len(group), world, caps)
    mine = [j for j, o in enumerate(own) if o == rank]
    if world == 1:
        return _Return([], result=rows)
    host = _via_host() and device.type != "cpu"
    if rank == src:
        ops, keep = [], []
        for r in range(world):
            idx = [j for j, o in enumerate(own) if o == r]
            if r == src or not idx:
                continue
            t = rows[idx].contiguous()
            t = t.cpu() if host else t
            keep.append(t)
            ops.append(dist.P2POp(dist.isend, t, r))
        return _Return(ops, result=rows[mine] if mine else rows[:0], keep=keep)
    shape, dtype = spec
    if not mine:
        return _Return([], result=torch.empty((0,) + tuple(shape), dtype=dtype, device=device))
    buf = torch.empty((len(mine),) + tuple(shape), dtype=dtype, device="cpu" if host else device)
    return _Return([dist.P2POp(dist.irecv, buf, src)], buf=buf, device=device)


class _Batch:
    """The works of one batch_isend_irecv, waited for at most once (a gloo work waited twice blocks forever), shared
    by the exchanges posted in it."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        works, self.works = self.works, []
        for w in works:
            w.wait()


def _post(ops) -> list:
    return [_Batch(dist.batch_isend_irecv(ops))] if ops else []


def run_pipeline(groups: Sequence[Sequence[int]], world: int, rank: int,
                 stylize: Callable[[List[int]], tuple],
                 root_post: Callable[[List[int], torch.Tensor], Optional[torch.Tensor]],
                 emit: Optional[Callable[[List[int], Optional[torch.Tensor], object], None]] = None,
                 ret_spec: Optional[Callable[[List[int]], tuple]] = None,
                 device: torch.device = torch.device("cpu"), caps: Optional[Sequence[int]] = None, root: int = 0):
    """Drive the sharded frame loop with an ordered stage on `root` and the output stage on each frame's owner.

    Per group: every rank stylizes its shard (`stylize(idx) -> (send, keep)`: `send` [len(idx), ...] goes to root for
    the ordered stage, `keep` stays with the owner); root runs `root_post(group, full)` on the whole group's `send`
    rows in frame order and returns per-frame rows [len(group), ...] (or None: nothing returns); each owner then
    gets its own rows back and runs `emit(idx, rows, keep)` (the D2H and the encode of its own frames).  A group's
    return leg and the next group's gather are posted as ONE batch of point-to-point ops (RCCL over every xGMI link
    at once), each completed one group later, so transfers overlap the next forward:

        iteration k: stylize(k) | finish return(k-2), emit(k-2) | finish gather(k-1), root_post(k-1) |
                     agree_ok | post return(k-1) + gather(k)

    `ret_spec(group) -> (per-frame shape, dtype)` of the returned rows (every rank must know it to post its receive).
    A failure anywhere (stylize, root_post, emit) reaches every rank through agree_ok before the next exchange: the
    failing rank re-raises its own error, the others raise RankFailed."""
    s_err = c_err = e_err = None
    pend_g = None   # (group, Exchange of the gather, keep)
    pend_r = None   # (group, _Return, keep)
    seq = list(groups) + [None, None]
    for g in seq:
        send = keep = None
        if g is not None and s_err is None:
            mine = shard(g, world, rank, caps)
            try:
                send, keep = stylize(mine)
            except Exception as e:  # noqa: BLE001 -- re-raised below on this rank
                s_err = e
        # the return leg posted last iteration: this rank's rows of group k-2 -> emit
        if pend_r is not None:
            pg, rex, pkeep = pend_r
            pend_r = None
            rows = rex.finish()
            if emit is not None and e_err is None:
                try:
                    emit(shard(pg, world, rank, caps), rows, pkeep)
                except Exception as e:  # noqa: BLE001
                    e_err = e
        # the gather posted last iteration: root runs the ordered stage of group k-1
        ret_post = None
        if pend_g is not None:
            pg, gex, pkeep = pend_g
            pend_g = None
            full = gather_finish(gex)
            ret = None
            if full is not None and c_err is None:
                try:
                    ret = root_post(list(pg), full)
                except Exception as e:  # noqa: BLE001
                    c_err = e
            ret_post = (pg, ret, pkeep)
        err = s_err or c_err or e_err
        if world > 1:
            agree_ok(err is None, device)
        if err is not None:
            raise err
        ops, rex, gex = [], None, None
        if ret_post is not None and ret_spec is not None:
            pg, ret, pkeep = ret_post
            spec = ret_spec(list(pg))
            if spec is not None:
                rex = return_ops(ret, pg, world, rank, spec, caps, root, device)
                ops += rex.ops
                pend_r = (pg, rex, pkeep)
        if g is not None:
            gex = gather_start(send, g, world, rank, caps, root, post=False)
            ops += gex.ops
            pend_g = (g, gex, keep)
        works = _post(ops)  # one batch: the return leg of group k-1 and the gather of group k
        for ex in (rex, gex):
            if ex is not None:
                ex.works = works


def run_sharded(groups: Sequence[Sequence[int]], world: int, rank: int,
                stylize: Callable[[List[int]], torch.Tensor], consume: Callable[[List[int], torch.Tensor], None],
                device: torch.device = torch.device("cpu"), caps: Optional[Sequence[int]] = None):
    """Gather-only form of run_pipeline: every rank stylizes its shard of each group, rank 0 consumes the group's
    frames in order (`consume(group, full)`); nothing returns to the owners."""
    run_pipeline(groups, world, rank, lambda idx: (stylize(idx), None),
                 lambda g, full: consume(g, full), None, None, device, caps)
