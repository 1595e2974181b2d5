"""Frame-parallel plumbing over torch.distributed (gloo, world_size 2, CPU).

Covers depth_pro.distributed: round-robin frame sharding, the one-blob packed
weight broadcast and the depth-map gather, exactly as bench.py / the frame loop
use them over RCCL on GPUs.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from depth_pro import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        packed = None
        if rank == 0:
            g = torch.Generator().manual_seed(0)
            packed = {"a.w": torch.randn(7, 5, generator=g).to(torch.bfloat16),
                      "b.b": torch.randn(13, generator=g),
                      "c.s": 0.25, "d.w": torch.randn(3, 64, generator=g).half()}
        got = D.broadcast_packed(packed, torch.device("cpu"), src=0)
        g = torch.Generator().manual_seed(0)
        ref = {"a.w": torch.randn(7, 5, generator=g).to(torch.bfloat16), "b.b": torch.randn(13, generator=g),
               "c.s": 0.25, "d.w": torch.randn(3, 64, generator=g).half()}
        ok_bcast = all((torch.equal(got[k], ref[k]) and got[k].dtype == ref[k].dtype) if torch.is_tensor(ref[k])
                       else got[k] == ref[k] for k in ref)
        frames = D.shard_frames(10, rank, world)
        per_step = []
        for k in frames[:4]:
            depth = torch.full((4, 6), float(k))  # stand-in for frame k's depth map
            out = D.gather_frames(depth, dst=0)
            if rank == 0:
                per_step.append(out)
        # bench.py's pattern: two output buffers, asynchronous gathers, a buffer rewritten
        # only after its previous gather's wait()
        bufs = [torch.empty(4, 6), torch.empty(4, 6)]
        pending, async_steps = [None, None], []
        for i, k in enumerate(frames[:4]):
            if pending[i & 1] is not None:
                pending[i & 1][1].wait()
                if rank == 0:
                    async_steps.append([t.clone() for t in pending[i & 1][0]])
            bufs[i & 1].fill_(float(k))
            pending[i & 1] = D.gather_frames(bufs[i & 1], dst=0, async_op=True)
        for j in (0, 1):
            pending[j][1].wait()
            if rank == 0:
                async_steps.append([t.clone() for t in pending[j][0]])
        if rank == 0:
            order = [int(t[0, 0].item()) for t in D.order_results(per_step, world)]
            q.put(("order", order))
            q.put(("async_order", [int(t[0, 0].item()) for t in D.order_results(async_steps, world)]))
        q.put(("rank", rank, frames, ok_bcast))
    finally:
        dist.destroy_process_group()


def test_frame_sharding_broadcast_gather_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=5) for _ in range(world + 2)]
    ranks = {m[1]: m for m in msgs if m[0] == "rank"}
    assert ranks[0][2] == [0, 2, 4, 6, 8] and ranks[1][2] == [1, 3, 5, 7, 9]
    assert ranks[0][3] and ranks[1][3]
    order = [m[1] for m in msgs if m[0] == "order"][0]
    assert order == list(range(8))  # stream order restored at rank 0
    assert [m[1] for m in msgs if m[0] == "async_order"][0] == list(range(8))


def test_shard_frames_covers_stream_once():
    for world in (1, 2, 3, 8):
        seen = sorted(k for r in range(world) for k in D.shard_frames(1024, r, world))
        assert seen == list(range(1024))
        assert all(D.frame_owner(k, world) == k % world for k in range(50))


class _StubModel:
    """Stands in for DepthPro in the frame loop: depth = a constant map tagged with the rank, so
    the test can see which rank produced each file."""

    def __init__(self, rank):
        self.rank = rank
        self.calls = []

    def infer(self, x, f_px=None):
        self.calls.append(int(x[0, 0, 0]))
        h, w = x.shape[-2:]
        d = torch.linspace(1.0, 2.0, h * w).reshape(h, w) + 10.0 * self.rank
        return {"depth": d, "focallength_px": torch.tensor(100.0)}


def _stub_transform(img):
    return torch.from_numpy(img).permute(2, 0, 1).float()


def _loop_worker(rank, world, port, src, out, resume, q):
    import generate_depth_maps as G

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stub = _StubModel(rank)
        n = G.batch_generate_depth_maps(src, out, pattern="output_*.png", model=(stub, _stub_transform),
                                        decode_workers=2, encode_workers=2, resume=resume)
        dist.barrier()
        q.put((rank, n, sorted(stub.calls)))
    finally:
        dist.destroy_process_group()


def _run_loop(world, src, out, resume):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_loop_worker, args=(r, world, port, src, out, resume, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return {m[0]: m[1:] for m in (q.get(timeout=5) for _ in range(world))}


def test_frame_loop_writes_every_frame_exactly_once_world2(tmp_path):
    """generate_depth_maps.batch_generate_depth_maps under a 2-rank gloo group with a stub engine:
    frame k is decoded and written by rank k mod 2 only, names follow the reference
    (`{base}_depth.png`), and --resume redoes exactly the missing frames."""
    from PIL import Image

    import numpy as np

    src, out = tmp_path / "frames", tmp_path / "depth"
    src.mkdir()
    for k in range(7):   # pixel (0,0) red channel = k: the stub records which frames it saw
        img = np.full((12, 16, 3), 50, dtype=np.uint8)
        img[0, 0, 0] = k
        Image.fromarray(img).save(src / f"output_{k:04d}.png")
    res = _run_loop(2, str(src), str(out), False)
    assert res[0][1] == [0, 2, 4, 6] and res[1][1] == [1, 3, 5]          # k -> rank k mod 2, once each
    assert res[0][0] + res[1][0] == 7
    files = sorted(os.listdir(out))
    assert files == [f"output_{k:04d}_depth.png" for k in range(7)]
    os.remove(out / "output_0003_depth.png")
    os.remove(out / "output_0004_depth.png")
    res2 = _run_loop(2, str(src), str(out), True)
    assert sorted(res2[0][1] + res2[1][1]) == [3, 4]                    # resume: only the missing frames
    assert res2[0][0] + res2[1][0] == 2
    assert sorted(os.listdir(out)) == files
