"""Frame-parallel execution over one process per GPU (torch.distributed / RCCL).

The video stream shards as independent frames: frame k runs on
rank k mod N, with no collective on the data path.  The collectives:
  * `broadcast_packed`: once at start-up rank 0 ships its packed (GEMM-ready,
    16-bit) weight set to every rank as ONE contiguous byte blob, so only rank 0
    reads/converts the checkpoint (one RCCL broadcast over xGMI);
    (`create_model_and_transforms_shared` wraps it for the frame loops);
  * `gather_frames`: per step, the depth maps travel to rank 0 (RCCL gather) --
    bench.py's stream; the directory loop writes each rank's frames locally;
  * the directory loop's resume list: rank 0 decides which frames still need work,
    one `broadcast_object_list` before any rank writes.
The same code runs over gloo on CPU tensors (tests/test_distributed.py).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_frames(n_frames: int, rank: int, world: int) -> List[int]:
    """Frame indices owned by `rank` (round-robin, frame k -> rank k mod world)."""
    return list(range(rank, n_frames, world))


def frame_owner(k: int, world: int) -> int:
    return k % world


def _layout(packed: Dict[str, object]):
    meta, off = [], 0
    for k in sorted(packed):
        v = packed[k]
        if torch.is_tensor(v):
            nbytes = v.numel() * v.element_size()
            meta.append((k, "t", str(v.dtype).replace("torch.", ""), tuple(v.shape), off, nbytes))
            off += (nbytes + 255) // 256 * 256
        else:
            meta.append((k, "f", float(v)))
    return meta, off


def broadcast_packed(packed: Optional[Dict[str, object]], device: torch.device, src: int = 0
                     ) -> Dict[str, object]:
    """Rank `src` passes its packed weight dict; every rank returns an identical dict on `device`."""
    rank = dist.get_rank()
    obj = [None]
    if rank == src:
        meta, total = _layout(packed)
        obj = [(meta, total)]
    dist.broadcast_object_list(obj, src=src)
    meta, total = obj[0]
    blob = torch.empty(total, dtype=torch.uint8, device=device)
    if rank == src:
        for m in meta:
            if m[1] == "t":
                k, _, _, _, off, nbytes = m
                blob[off:off + nbytes].copy_(packed[k].contiguous().view(-1).view(torch.uint8))
    dist.broadcast(blob, src=src)
    out: Dict[str, object] = {}
    for m in meta:
        if m[1] == "t":
            k, _, dt, shape, off, nbytes = m
            out[k] = blob[off:off + nbytes].view(getattr(torch, dt)).view(shape)
        else:
            out[m[0]] = m[2]
    return out


def create_model_and_transforms_shared(config, device: torch.device, precision: torch.dtype = torch.float32,
                                       src: int = 0):
    """`create_model_and_transforms` for a process group: only rank `src` reads the checkpoint
    and packs it (depth_pro.py:134-149 + engine.pack_weights); the packed 16-bit weight set
    reaches every other rank as one RCCL broadcast (`broadcast_packed`), which builds its
    engine on it directly (DepthPro.from_packed).  Every rank of the group must call this."""
    from .depth_pro import DepthPro, Transform, create_model_and_transforms

    rank = dist.get_rank()
    info = [None]
    packed = None
    if rank == src:
        model, transform = create_model_and_transforms(config, device=device, precision=precision)
        packed = model.engine().P
        info = [(model.use_fov_head, tuple(model.compute_dtype))]
    dist.broadcast_object_list(info, src=src)
    received = broadcast_packed(packed, device, src=src)
    if rank == src:
        del received           # rank src keeps the engine it packed
        return model, transform
    use_fov, codes = info[0]
    return DepthPro.from_packed(received, device, codes, use_fov_head=use_fov), Transform(device, precision)


def gather_frames(t: torch.Tensor, dst: int = 0, async_op: bool = False):
    """Gather one equally-shaped tensor per rank to `dst` (rank order).

    async_op=True returns (bufs, work): the gather runs on the collective's own
    stream while the caller queues the next frame; `work.wait()` (which makes the
    current stream, not the host, wait under RCCL) must precede any reuse of `t`
    or read of `bufs`.
    """
    world, rank = dist.get_world_size(), dist.get_rank()
    if world == 1:
        return ([t], None) if async_op else [t]
    bufs = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
    work = dist.gather(t, gather_list=bufs, dst=dst, async_op=async_op)
    return (bufs, work) if async_op else bufs


def order_results(per_step: Sequence[Sequence[torch.Tensor]], world: int) -> List[torch.Tensor]:
    """Flatten [step][rank] gathered frames back into stream order k = step*world + rank."""
    out = []
    for step in per_step:
        out.extend(step[:world])
    return out
