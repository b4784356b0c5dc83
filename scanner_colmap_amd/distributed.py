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

    Sizes are exchanged with an all_gather of one int64 per rank; then ONE
    batch_isend_irecv group moves every rank's exact payload to rank 0 (no
    padding): rank r > 0 posts its send, rank 0 posts all receives at once into
    views of one flat buffer.  On the `nccl` backend (RCCL over xGMI) the
    group is device-resident end to end -- each sender stages its payload once
    host -> device (the library's io.cc rows live in pinned host memory), each
    peer's bytes travel over its own xGMI link to GPU 0, and rank 0 copies the
    flat buffer to the host once; on gloo the same group runs on CPU tensors."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    src = (np.frombuffer(payload, dtype=np.uint8) if isinstance(payload, (bytes, bytearray))
           else np.ascontiguousarray(payload, dtype=np.uint8).reshape(-1))
    n = torch.tensor([src.size], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank != 0:
        if sizes[rank]:
            host = torch.from_numpy(src if src.flags.writeable else src.copy())
            t = host.to(dev, non_blocking=False) if dev.type != "cpu" else host
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 0)]):
                w.wait()
        return None
    offs = np.concatenate([[0], np.cumsum(sizes[1:])]).astype(np.int64)
    flat = torch.empty(int(offs[-1]), dtype=torch.uint8, device=dev)
    ops = [dist.P2POp(dist.irecv, flat[int(offs[r - 1]):int(offs[r])], r)
           for r in range(1, world) if sizes[r]]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    host = flat.cpu().numpy() if dev.type != "cpu" else flat.numpy()
    out = [src.tobytes()]
    for r in range(1, world):
        out.append(host[int(offs[r - 1]):int(offs[r])].tobytes())
    return out


class ShardPlan:
    """One rank's share of a sequential-matching job (bench.py and the job
    script use this; tests/test_distributed.py drives it over gloo).

    weak scaling: every rank owns `images` pivot rows of one long sequence
    (total = images * world); strong: `images` rows in total, split over the
    ranks (BASELINE configs 4 and 5).  Rows are balanced by pair count and a
    rank loads its rows plus the overlap-1 halo."""

    def __init__(self, images: int, overlap: int, world: int, rank: int, scaling: str = "weak"):
        if scaling not in ("weak", "strong"):
            raise ValueError(f"scaling must be weak or strong, got {scaling!r}")
        self.overlap = overlap
        self.world = world
        self.rank = rank
        self.total_images = images if scaling == "strong" else images * world
        self.row_begin, self.row_end = shard_rows(self.total_images, overlap, world, rank)
        self.table_begin, self.table_end = table_range(self.row_begin, self.row_end,
                                                       self.total_images, overlap)

    @property
    def local_rows(self) -> tuple[int, int]:
        """The rank's output rows as indices into its loaded table slice."""
        return self.row_begin - self.table_begin, self.row_end - self.table_begin

    def pairs(self) -> int:
        return int(pairs_per_row(self.total_images, self.overlap)[self.row_begin:self.row_end].sum())

    def step(self, runner, device=None):
        """One pass of the op over this rank's rows: `runner.table_run_packed`
        (the scm_table_run_packed binding, or a stand-in with the same
        result shape), then for world > 1 the gather of the packed io.cc rows
        to rank 0.  Returns (this rank's packed rows, the gathered per-rank
        payloads on rank 0 / None)."""
        lb, le = self.local_rows
        packed = runner.table_run_packed(self.overlap, lb, le)
        gathered = None
        if self.world > 1:
            gathered = gather_to_root(pack_packed(packed.offsets, packed.data), device=device)
        return packed, gathered


def merge_gathered(payloads: list) -> tuple[list[bytes], list[bytes]]:
    """Rank 0: concatenate the gathered per-rank packed rows in rank order
    (= pivot-row order) into (pair_image_ids rows, two_view_geometries rows)."""
    rows_a, rows_b = [], []
    for p in payloads:
        if len(p) == 0:
            continue
        a, b = unpack_packed(p)
        rows_a += a
        rows_b += b
    return rows_a, rows_b
