"""Host-side logic on CPU: CLI parity, sharding + ordered gather (gloo, world 2), env adapter."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from neuralstyletransferv1_amd import frames as F
from neuralstyletransferv1_amd import pipeline as P
from neuralstyletransferv1_amd import run_videos as RV


def test_cli_has_every_reference_flag():
    ref = json.load(open(os.path.join(GOLDEN, "reference_flags.json")))["flags"]
    ours = {a for act in P.build_parser()._actions for a in act.option_strings}
    missing = [f for f in ref if f not in ours]
    assert not missing, missing


def test_cli_defaults_match_reference():
    a = P.build_parser().parse_args([])
    assert (a.smooth_lightness, a.smooth_alpha, a.blend, a.io_preset, a.image_ext, a.jpeg_quality, a.threads,
            a.composite_mode, a.fit_mask_to, a.model_type, a.chroma_alpha) == (
        True, 0.7, 1.0, "auto", "png", 85, 4, "keep", "input", "transformer", 0.85)


@pytest.mark.parametrize("extra", [["--model_type", "magenta"], ["--model_type", "torch7"], ["--device", "cpu"]])
def test_out_of_scope_requests_fail_loudly(extra, tmp_path):
    args = P.build_parser().parse_args(["--model", "x.pth", "--synthetic", "64x48"] + extra)
    with pytest.raises(SystemExit) as e:
        P.prepare(args)
    assert e.value.code == 2


def test_parse_blend_weights():
    assert P.parse_blend_weights(None, 4) == [0.25] * 4
    assert P.parse_blend_weights("0.5,0.5", 2) == [0.5, 0.5]
    with pytest.raises(ValueError):
        P.parse_blend_weights("0.5,0.6", 2)
    with pytest.raises(ValueError):
        P.parse_blend_weights("1.0", 2)


def test_plan_groups_and_round_robin_shard():
    sizes = [(4, 4)] * 5 + [(8, 8)] * 3
    g = F.plan_groups(sizes, world=2, batch=2)
    assert g == [[0, 1, 2, 3], [4], [5, 6, 7]]
    assert F.shard(g[0], 2, 0) == [0, 2] and F.shard(g[0], 2, 1) == [1, 3]
    assert F.shard([4], 2, 1) == []


def test_owners_with_caps():
    """owners(): round-robin over the ranks that still have room (rank 0's lighter share, frames.rank0_share)."""
    assert F.owners(5, 2) == [0, 1, 0, 1, 0]
    assert F.owners(5, 2, [1, 4]) == [0, 1, 1, 1, 1]
    assert F.owners(7, 3, [1, 3, 3]) == [0, 1, 2, 1, 2, 1, 2]
    assert F.owners(3, 3, [1, 3, 3]) == [0, 1, 2]  # a short last group: every rank's first slot in order
    assert F.owners(2, 3, [0, 3, 3]) == [1, 2]
    with pytest.raises(ValueError):
        F.owners(8, 3, [1, 3, 3])
    for world, batch in ((2, 8), (3, 8), (8, 8), (8, 2)):
        caps = [F.rank0_share(world, batch)] + [batch] * (world - 1)
        own = F.owners(sum(caps), world, caps)
        assert [own.count(r) for r in range(world)] == caps
    assert F.rank0_share(8, 8) == 6 and F.rank0_share(1, 8) == 8
    g = F.plan_groups([(4, 4)] * 9 + [(8, 8)] * 2, world=2, batch=3, rank0_batch=1)
    assert g == [[0, 1, 2, 3], [4, 5, 6, 7], [8], [9, 10]]


def _gather_worker(rank, world, port, q, caps=None):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    seen = []
    groups = F.plan_groups([(2, 3)] * 7 + [(5, 1)] * 2, world, batch=2 if caps is None else caps[1],
                           rank0_batch=None if caps is None else caps[0])

    def stylize(idx):
        if not idx:
            return torch.empty((0, 2, 3, 3), dtype=torch.uint8)
        h, w = (2, 3) if idx[0] < 7 else (5, 1)
        return torch.stack([torch.full((h, w, 3), f, dtype=torch.uint8) for f in idx])

    def consume(g, full):
        seen.append((g, [int(full[j].flatten()[0]) for j in range(full.shape[0])]))

    F.run_sharded(groups, world, rank, stylize, consume, caps=caps)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, seen))


@pytest.mark.parametrize("world,caps", [(2, None), (3, None), (2, [1, 3]), (3, [1, 2, 2]), (3, [2, 3, 3])])
def test_ordered_gather_gloo(world, caps):
    """Frames come back to rank 0 in order: equal shares, and the pipeline's caps (rank 0 lighter) with a short
    last group and a frame-size change (7 frames of one size, then 2 of another)."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, caps)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    seen0 = res[0]
    assert all(not res[r] for r in range(1, world))
    flat = [f for g, vals in seen0 for f in g]
    assert flat == list(range(9))
    for g, vals in seen0:
        assert vals == g  # frame j of each group is the frame itself, in order


def _pipeline_worker(rank, world, port, q, caps=None, fail_emit=None):
    """run_pipeline with an ordered stage on rank 0 (a running sum over the frames in order, like the LAB EMA's
    state) and the output stage on each frame's owner."""
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sizes = [(2, 3)] * 7 + [(5, 1)] * 4
    groups = F.plan_groups(sizes, world, batch=2 if caps is None else caps[1],
                           rank0_batch=None if caps is None else caps[0])
    emitted, state = [], [0]

    def stylize(idx):
        h, w = sizes[idx[0]] if idx else sizes[0]
        send = torch.stack([torch.full((h * w,), f + 1, dtype=torch.int64) for f in idx]) if idx else \
            torch.empty((0, h * w), dtype=torch.int64)
        return send, [f * 10 for f in idx]

    def root_post(g, full):
        out = []
        for j in range(full.shape[0]):  # sequential: frame j's value depends on every earlier frame
            state[0] += int(full[j, 0])
            out.append(torch.full_like(full[j], state[0]))
        return torch.stack(out)

    def emit(idx, rows, keep):
        if fail_emit is not None and rank == fail_emit and idx and idx[0] >= 4:
            raise OSError("encode failed")
        assert keep == [f * 10 for f in idx] and rows.shape[0] == len(idx)
        emitted.extend((f, int(rows[j, 0]), rows.shape[1]) for j, f in enumerate(idx))

    outcome = "ok"
    try:
        F.run_pipeline(groups, world, rank, stylize, root_post, emit,
                       lambda g: ((sizes[g[0]][0] * sizes[g[0]][1],), torch.int64), caps=caps)
    except F.RankFailed:
        outcome = "RankFailed"
    except OSError:
        outcome = "OSError"
    dist.destroy_process_group()
    q.put((rank, outcome, emitted, [F.shard(g, world, rank, caps) for g in groups]))


@pytest.mark.parametrize("world,caps", [(2, None), (3, None), (3, [1, 2, 2])])
def test_pipeline_returns_each_frame_to_its_owner(world, caps):
    """Multi-GPU output leg: rank 0 runs the ordered stage over the group's frames in order and
    sends each frame's result back to the rank that stylized it; each rank emits (D2H + encode) exactly its own
    frames, with the values the single-rank sequential order gives; a frame-size change mid-stream."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, q, caps)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (o, e, sh) for r, o, e, sh in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    expect = np.cumsum(np.arange(1, 12))
    sizes = [6] * 7 + [5] * 4
    seen = set()
    for r in range(world):
        outcome, emitted, shards = res[r]
        assert outcome == "ok"
        assert [f for f, _, _ in emitted] == [f for sh in shards for f in sh]  # only its own frames, in order
        for f, v, n in emitted:
            assert v == expect[f] and n == sizes[f], (r, f, v)
            seen.add(f)
    assert seen == set(range(11))


def test_pipeline_emit_failure_reaches_every_rank():
    """An owner whose output stage raises (disk full) stops every rank."""
    import torch.multiprocessing as mp
    world = 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, q, None, 1)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: o for r, o, _, _ in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "RankFailed", 1: "OSError", 2: "RankFailed"}


def _failing_worker(rank, world, port, fail_rank, fail_in, q, caps=None):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    groups = F.plan_groups([(2, 3)] * 8, world, batch=2, rank0_batch=None if caps is None else caps[0])
    consumed = []

    def stylize(idx):
        if fail_in == "stylize" and rank == fail_rank and idx and idx[0] >= 4:
            raise ValueError("bad frame")
        if not idx:
            return torch.empty((0, 2, 3, 3), dtype=torch.uint8)
        return torch.stack([torch.full((2, 3, 3), f, dtype=torch.uint8) for f in idx])

    def consume(g, full):
        if fail_in == "consume" and g[0] >= 4:
            raise OSError("disk full")
        consumed.append(list(g))

    try:
        F.run_sharded(groups, world, rank, stylize, consume, caps=caps)
        outcome = "ok"
    except F.RankFailed:
        outcome = "RankFailed"
    except (ValueError, OSError) as e:
        outcome = type(e).__name__
    dist.destroy_process_group()
    q.put((rank, outcome, consumed))


@pytest.mark.parametrize("fail_in,fail_rank,caps", [("stylize", 1, None), ("stylize", 0, None), ("consume", 0, None),
                                                    ("stylize", 2, [1, 2, 2]), ("consume", 0, [1, 2, 2])])
def test_sharded_failure_reaches_every_rank(fail_in, fail_rank, caps):
    """A rank whose stylize (or rank 0 whose consume) raises must not leave the others blocked in the
    point-to-point exchange: every rank stops (the failing one with its own error); also with rank 0's lighter
    share (caps: groups of 5 frames, 1 of them on rank 0)."""
    import torch.multiprocessing as mp
    world = 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, fail_rank, fail_in, q, caps))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (o, c) for r, o, c in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
    own = "ValueError" if fail_in == "stylize" else "OSError"
    for r in range(world):
        assert res[r][0] == (own if r == fail_rank else "RankFailed"), (r, res[r])
    # the group before the failure was consumed, nothing after (groups of 6 frames; 5 with caps [1, 2, 2], where
    # the failing group is [5..7], whose frames >= 4 fail on every rank holding one)
    assert res[0][1] == ([[0, 1, 2, 3, 4, 5]] if caps is None else [[0, 1, 2, 3, 4]])


def test_run_videos_env_mapping(monkeypatch):
    for k in list(os.environ):
        if k.startswith(("MODEL_", "IO_PRESET", "BLEND", "GPUS", "SMOOTH", "MAX_FRAMES")):
            monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MODEL_A", "/m/candy.pth")
    monkeypatch.setenv("MODEL_B", "mosaic")
    monkeypatch.setenv("MODEL_B_TYPE", "pytorch")
    monkeypatch.setenv("IO_PRESET", "raw_255")
    monkeypatch.setenv("BLEND_WEIGHTS", "0.7,0.3")
    monkeypatch.setenv("GPUS", "4")
    monkeypatch.setenv("MAX_FRAMES", "10")
    cmd = RV.build_pipeline_cmd("/in/clip.mp4")
    s = " ".join(cmd)
    assert "--model /m/candy.pth --model_type transformer --io_preset raw_255" in s
    assert "--model_b /app/models/pytorch/mosaic.pth --model_b_type transformer" in s
    assert "--blend_models_weights 0.7,0.3" in s and "--gpus 4" in s and "--max_frames 10" in s
    assert "--smooth_alpha 0.65" in s and "--blend 0.9" in s and "--scale 720" in s
    args = P.build_parser().parse_args(cmd[3:])  # the pipeline accepts the adapter's command line
    assert args.gpus == 4 and args.model_b.endswith("mosaic.pth")


def test_mask_fit_matches_oracle():
    from oracle import nst_oracle as O
    for m in ("center_circle.png", "gradient_horizontal.png"):
        path = os.path.join(GOLDEN, "masks", m)
        for hw, inv in (((96, 128), False), ((128, 96), True), ((50, 50), False)):
            ours = P.load_mask_fit(path, hw, inv)
            ref = O.load_mask_fit(path, hw, inv)[..., 0]
            assert np.array_equal(ours, ref)


def test_lab_weight_rules_match_reference():
    """pipeline.py:1843-1852 weight rules for the LAB blend, host mirror vs oracle restatement."""
    from oracle import nst_oracle as O
    for s, n in ((None, 2), (None, 3), (None, 5), ("0.3,0.7", 3), ("0.2,0.3,0.5", 4), ("0.1,0.2,0.3,0.4", 5)):
        assert P.lab_weights_rest(s, n) == O.lab_weights_rest(s, n)
    assert P.lab_weights_rest("0.1,0.2,0.3,0.4", 5) == [0.25] * 4  # the reference's length rule
    assert P.parse_lab_weights(None) == (0.5, 0.5) and P.parse_lab_weights("0.3,0.7") == (0.3, 0.7)
    with pytest.raises(ValueError):
        P.parse_lab_weights("0.3,0.8")


def test_feather_restatement_properties():
    """Oracle feather (parity unpinned): symmetric kernel, constant image fixed, radius rule."""
    import numpy as np
    from oracle import nst_oracle as O
    m = np.full((20, 30), 77, np.uint8)
    assert np.array_equal(O.feather_mask_u8(m, 8), m)
    m = np.zeros((31, 31), np.uint8)
    m[15, 15] = 255
    f = O.feather_mask_u8(m, 4).astype(int)
    assert np.array_equal(f, f[::-1, ::-1]) and np.array_equal(f, f.T)


def test_check_scratch_flags_spills(tmp_path):
    """tools/check_scratch.py (run by the Makefile on the counted-vmcnt kernels): a kernel with scratch fails the
    build (NST_STRICT_SCRATCH=0 only reports it), a clean remarks file passes, compiler warnings are echoed."""
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    rem = "x.hip:1:1: remark: {} [-Rpass-analysis=kernel-resource-usage]\n"
    ok = tmp_path / "ok.rem"
    ok.write_text(rem.format("Function Name: k0") + "    1 | __global__ void k0()\n      | ^\n"
                  + rem.format("    ScratchSize [bytes/lane]: 0") + "x.hip:2:1: warning: unused\n")
    bad = tmp_path / "bad.rem"
    bad.write_text(rem.format("Function Name: k1") + rem.format("    ScratchSize [bytes/lane]: 20"))
    r = subprocess.run([sys.executable, str(root / "tools/check_scratch.py"), str(ok)], capture_output=True, text=True)
    assert r.returncode == 0 and "warning: unused" in r.stderr and "__global__" not in r.stderr
    env = {k: v for k, v in os.environ.items() if k != "NST_STRICT_SCRATCH"}
    r = subprocess.run([sys.executable, str(root / "tools/check_scratch.py"), str(bad)], capture_output=True, text=True,
                       env=env)
    assert r.returncode == 1 and "k1 uses 20 bytes/lane" in r.stderr
    r = subprocess.run([sys.executable, str(root / "tools/check_scratch.py"), str(bad)], capture_output=True, text=True,
                       env=dict(env, NST_STRICT_SCRATCH="0"))
    assert r.returncode == 0


@pytest.mark.parametrize("shape", [(1, 1, 3), (1, 7, 3), (5, 1, 3), (37, 53, 3), (64, 96, 4), (33, 17)])
def test_fast_png_writer_decodes_to_the_same_pixels(shape, tmp_path):
    """pngio.encode_png (Up filter + zlib RLE; the CLI's default PNG writer) decodes with Pillow to exactly the
    array it was given: noise, flat and ramp content, RGB / RGBA / grey, one-pixel rows and columns."""
    from PIL import Image
    from neuralstyletransferv1_amd import pngio
    rng = np.random.default_rng(sum(shape))
    for kind in ("noise", "flat", "ramp"):
        if kind == "noise":
            a = rng.integers(0, 256, size=shape, dtype=np.uint8)
        elif kind == "flat":
            a = np.full(shape, 200, np.uint8)
        else:
            a = (np.arange(int(np.prod(shape))) % 251).astype(np.uint8).reshape(shape)
        p = tmp_path / f"{kind}.png"
        pngio.write_png(p, a)
        with Image.open(p) as im:
            assert im.size == (shape[1], shape[0])
            got = np.array(im)
        assert got.dtype == np.uint8 and np.array_equal(got, a), kind
    with pytest.raises(ValueError):
        pngio.encode_png(np.zeros((4, 4, 3), np.float32))
