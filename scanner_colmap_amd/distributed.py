"""Multi-GPU plumbing: pair-balanced row sharding and the RCCL gather of the
output rows.

One process per GPU.  Image pairs are independent, so ranks own contiguous
pivot-row ranges (plus the overlap-1 halo rows their stencils read) and run
with no collective in the data path; the only exchange is gathering the
io.cc-encoded `pair_image_ids` / `two_view_geometries` rows to rank 0 —
RCCL over xGMI when the process group is `nccl`, gloo on CPU in the tests.
"""
from __future__ import annotations

import struct

import numpy as np


def pairs_per_row(num_rows: int, overlap: int) -> np.ndarray:
    """Pairs emitted by each output row of the stencil range(0, overlap)
    (feature_matching.py:43): row i pairs with i+1 .. min(i+overlap-1, N-1)
    (distinct image ids assumed)."""
    i = np.arange(num_rows)
    return np.minimum(overlap - 1, num_rows - 1 - i).clip(min=0)


def shard_rows(num_rows: int, overlap: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous output-row range of `rank`, balanced by pair count."""
    if world <= 1:
        return 0, num_rows
    c = np.concatenate([[0], np.cumsum(pairs_per_row(num_rows, overlap))])
    total = c[-1]
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(np.searchsorted(c, total * r / world, side="left")))
    bounds.append(num_rows)
    bounds = np.maximum.accumulate(np.array(bounds))
    return int(bounds[rank]), int(bounds[rank + 1])


def table_range(row_begin: int, row_end: int, num_rows: int, overlap: int) -> tuple[int, int]:
    """Table rows a shard must load: its rows plus the overlap-1 halo."""
    return row_begin, min(num_rows, row_end + overlap - 1)


def pack_rows(pair_blobs: list[bytes], tvg_blobs: list[bytes]) -> bytes:
    parts = [struct.pack("<Q", len(pair_blobs))]
    for a, b in zip(pair_blobs, tvg_blobs):
        parts.append(struct.pack("<QQ", len(a), len(b)))
        parts.append(a)
        parts.append(b)
    return b"".join(parts)


def unpack_rows(buf: bytes) -> tuple[list[bytes], list[bytes]]:
    (n,) = struct.unpack_from("<Q", buf, 0)
    off = 8
    pa, pb = [], []
    for _ in range(n):
        la, lb = struct.unpack_from("<QQ", buf, off)
        off += 16
        pa.append(bytes(buf[off:off + la]))
        off += la
        pb.append(bytes(buf[off:off + lb]))
        off += lb
    return pa, pb


def gather_to_root(payload: bytes, device=None) -> list[bytes] | None:
    """Gather every rank's byte payload to rank 0 (None elsewhere).

    Sizes are exchanged with an all_gather of one int64 per rank, then each
    rank ships its payload (padded to the largest) with dist.gather — on the
    `nccl` (RCCL) backend every peer sends over its own xGMI link."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(1, max(sizes))
    t = torch.zeros(mx, dtype=torch.uint8, device=dev)
    if payload:
        t[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    bufs = [torch.zeros(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=bufs, dst=0)
    if rank != 0:
        return None
    return [bytes(b[:s].cpu().numpy().tobytes()) for b, s in zip(bufs, sizes)]
