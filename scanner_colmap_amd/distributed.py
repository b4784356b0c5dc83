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
        target = total * r / world
        k = int(np.searchsorted(c, target, side="left"))  # first cut with c[k] >= target
        if k > 0 and target - c[k - 1] < c[min(k, num_rows)] - target:
            k -= 1  # the cut before it is closer to the ideal split
        bounds.append(k)
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


def pack_packed(offsets: np.ndarray, data: np.ndarray) -> np.ndarray:
    """Payload of one rank's scm_table_run_packed output: element count,
    the 2n+1 element offsets, then the packed element bytes."""
    offs = np.ascontiguousarray(offsets, dtype=np.int64)
    head = np.array([offs.size], dtype=np.int64)
    return np.concatenate([head.view(np.uint8), offs.view(np.uint8),
                           np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)])


def unpack_packed(buf) -> tuple[list[bytes], list[bytes]]:
    """Inverse of pack_packed, split into (pair_image_ids, tvgs) rows."""
    b = np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, (bytes, bytearray)) else buf
    (n,) = b[:8].view(np.int64)
    offs = b[8:8 + 8 * n].view(np.int64)
    data = b[8 + 8 * n:]
    rows = (n - 1) // 2
    pa = [data[offs[2 * r]:offs[2 * r + 1]].tobytes() for r in range(rows)]
    pb = [data[offs[2 * r + 1]:offs[2 * r + 2]].tobytes() for r in range(rows)]
    return pa, pb


def gather_to_root(payload, device=None) -> list[bytes] | None:
    """Gather every rank's byte payload (bytes or a uint8 numpy array) to
    rank 0 (None elsewhere).

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
    if len(payload):
        src = (np.frombuffer(payload, dtype=np.uint8) if isinstance(payload, (bytes, bytearray))
               else np.ascontiguousarray(payload, dtype=np.uint8).reshape(-1))
        t[: len(payload)] = torch.from_numpy(src.copy() if not src.flags.writeable else src).to(dev)
    bufs = [torch.zeros(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gather_list=bufs, dst=0)
    if rank != 0:
        return None
    return [bytes(b[:s].cpu().numpy().tobytes()) for b, s in zip(bufs, sizes)]
