"""Multi-GPU plumbing: pair-balanced row sharding and the RCCL gather of the
output rows.

One process per GPU.  Image pairs are independent, so ranks own contiguous
pivot-row ranges (plus the overlap-1 halo rows their stencils read) and run
with no collective in the data path; the only exchange is gathering the
io.cc-encoded `pair_image_ids` / `two_view_geometries` rows to rank 0 —
RCCL over xGMI when the process group is `nccl`, gloo on CPU in the tests.
"""
from __future__ import annotations

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


class _Staging:
    """Persistent transfer buffers of the nccl gather (grown, never shrunk):
    a pinned host buffer and a device buffer for the sender's H2D hop, and a
    ring of two pinned host buffers for rank 0's D2H (a gather's views stay
    valid until the gather after next)."""

    def __init__(self):
        self.pin = None
        self.dev = None
        self.ring = [None, None]
        self.k = 0

    @staticmethod
    def _grow(buf, n, **kw):
        import torch
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(n, 1 << 20), dtype=torch.uint8, **kw)
        return buf

    def send_buffers(self, n, device):
        self.pin = self._grow(self.pin, n, pin_memory=True)
        self.dev = self._grow(self.dev, n, device=device)
        return self.pin, self.dev

    def recv_host(self, n):
        self.k ^= 1
        self.ring[self.k] = self._grow(self.ring[self.k], n, pin_memory=True)
        return self.ring[self.k]


def gather_packed(offsets: np.ndarray, data: np.ndarray, device=None, staging=None,
                  own: bool = False):
    """Gather every rank's scm_table_run_packed output (element offsets and
    packed element bytes) to rank 0: a list of (offsets int64 array, data
    uint8 array) per rank on rank 0, None elsewhere.

    Sizes travel in one all_gather (two int64 per rank); then ONE
    batch_isend_irecv group moves each rank's offsets and bytes to rank 0 as
    two messages (no packing copy), rank 0 posting every receive at once into
    slices of one flat buffer.  On `nccl` (RCCL over xGMI) a sender stages its
    bytes into a persistent pinned buffer and one H2D copy, each peer's bytes
    travel over its own xGMI link to GPU 0, and rank 0 makes one D2H copy into
    a pinned ring buffer; the per-rank results are views into it, valid until
    the gather after next.  `own`: results that outlive that (a kept
    background gather) -- rank 0's D2H lands in a buffer of their own instead
    of the ring.  Rank 0's own entry is a view of `data` (a PackedRows buffer
    lives as long as its views).  On gloo the same group runs on CPU tensors
    with no staging."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = device if device is not None else torch.device("cpu")
    on_gpu = dev.type != "cpu"
    offs = np.ascontiguousarray(offsets, dtype=np.int64).reshape(-1)
    dat = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    ob = offs.view(np.uint8)
    meta = torch.tensor([[ob.size, dat.size]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, 2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, meta)
    sizes = [tuple(int(x) for x in t.cpu().view(-1)) for t in sizes]
    if rank != 0:
        no, nd = sizes[rank]
        if no + nd == 0:
            return None
        if on_gpu:
            pin, dbuf = (staging or _Staging()).send_buffers(no + nd, dev)
            hp = pin.numpy()
            hp[:no] = ob
            hp[no:no + nd] = dat
            dbuf[:no + nd].copy_(pin[:no + nd], non_blocking=True)
            t_o, t_d = dbuf[:no], dbuf[no:no + nd]
        else:
            t_o, t_d = torch.from_numpy(ob), torch.from_numpy(dat if dat.flags.writeable else dat.copy())
        ops = [dist.P2POp(dist.isend, t, 0) for t in (t_o, t_d) if t.numel()]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if on_gpu:
            # wait() orders the stream only: the staging buffers are reused by
            # the next gather, so the copy and the sends must be complete
            torch.cuda.current_stream(dev).synchronize()
        return None
    starts = np.concatenate([[0], np.cumsum([a + b for a, b in sizes[1:]])]).astype(np.int64)
    total = int(starts[-1])
    flat = torch.empty(total, dtype=torch.uint8, device=dev)
    ops = []
    for r in range(1, world):
        a, no, nd = int(starts[r - 1]), sizes[r][0], sizes[r][1]
        if no:
            ops.append(dist.P2POp(dist.irecv, flat[a:a + no], r))
        if nd:
            ops.append(dist.P2POp(dist.irecv, flat[a + no:a + no + nd], r))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if on_gpu and total:
        if own or staging is None:
            host_t = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        else:
            host_t = staging.recv_host(total)
        host_t[:total].copy_(flat)
        host = host_t.numpy()
    else:
        host = flat.numpy()
    out = [(offs, dat)]
    for r in range(1, world):
        a, no, nd = int(starts[r - 1]), sizes[r][0], sizes[r][1]
        out.append((host[a:a + no].view(np.int64), host[a + no:a + no + nd]))
    return out


class Gatherer:
    """Runs gather_packed on a background thread, one gather at a time in step
    order, so that step k's rows travel to rank 0 while step k + 1 computes.
    At most two gathers are outstanding (submit waits for the older one)."""

    def __init__(self, device=None):
        from concurrent.futures import ThreadPoolExecutor
        self.device = device
        self.pool = ThreadPoolExecutor(max_workers=1)
        self.pending = []
        self.done = []  # results of the gathers already waited for, in step order
        self.staging = _Staging()
        self.ms = []  # duration of each gather (ms)

    def _run(self, packed, keep):
        import time
        if self.device is not None and self.device.type == "cuda":
            import torch
            torch.cuda.set_device(self.device)
        t0 = time.perf_counter()
        out = gather_packed(packed.offsets, packed.data, self.device, self.staging, own=keep)
        self.ms.append((time.perf_counter() - t0) * 1e3)
        return out

    def submit(self, packed, keep: bool = True):
        while len(self.pending) >= 2:
            f, k = self.pending.pop(0)
            r = f.result()
            if k:
                self.done.append(r)
        self.pending.append((self.pool.submit(self._run, packed, keep), keep))

    def drain(self) -> list:
        """Wait for every outstanding gather; the kept results in step order
        (each in buffers of its own: valid for as long as the caller keeps it)."""
        for f, k in self.pending:
            r = f.result()
            if k:
                self.done.append(r)
        out, self.done, self.pending = self.done, [], []
        return out


# Chunk header flags (the third int64 of a chunk header).
CHUNK_DATA, CHUNK_END, CHUNK_ERROR = 0, 1, 2


class ChunkSender:
    """rank != 0 of a chunked step: each chunk's packed rows (a batch of the
    library's pipeline, scm_table_run_chunks) go to rank 0 from a background
    thread while the next batches compute, in order: a header (offset bytes,
    data bytes, flag) and the two messages, one batch_isend_irecv group per
    chunk (RCCL over xGMI on nccl, staged through the same pinned / device
    buffers as gather_packed; gloo on CPU tensors).  The last header carries
    CHUNK_END, or CHUNK_ERROR when this rank's run failed (finish(error=True)):
    rank 0 then raises instead of waiting for rows that will not come."""

    def __init__(self, device=None):
        from concurrent.futures import ThreadPoolExecutor
        self.device = device
        self.pool = ThreadPoolExecutor(max_workers=1)
        self.futs = []
        self.staging = _Staging()

    def _send(self, offsets, data, flag):
        import torch
        import torch.distributed as dist
        dev = self.device if self.device is not None else torch.device("cpu")
        on_gpu = dev.type != "cpu"
        if on_gpu:
            torch.cuda.set_device(dev)
        ob = np.ascontiguousarray(offsets, dtype=np.int64).reshape(-1).view(np.uint8)
        dat = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
        no, nd = (0, 0) if flag != CHUNK_DATA else (ob.size, dat.size)
        hdr = torch.tensor([no, nd, flag], dtype=torch.int64, device=dev)
        ops = [dist.P2POp(dist.isend, hdr, 0)]
        if no + nd:
            if on_gpu:
                pin, dbuf = self.staging.send_buffers(no + nd, dev)
                hp = pin.numpy()
                hp[:no] = ob
                hp[no:no + nd] = dat
                dbuf[:no + nd].copy_(pin[:no + nd], non_blocking=True)
                t_o, t_d = dbuf[:no], dbuf[no:no + nd]
            else:
                t_o = torch.from_numpy(ob.copy())
                t_d = torch.from_numpy(dat.copy())
            ops += [dist.P2POp(dist.isend, t, 0) for t in (t_o, t_d) if t.numel()]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if on_gpu:
            torch.cuda.current_stream(dev).synchronize()  # staging reused by the next chunk

    def submit(self, packed):
        self.futs.append(self.pool.submit(self._send, packed.offsets, packed.data, CHUNK_DATA))

    def finish(self, error: bool = False):
        """Sends the end marker (CHUNK_ERROR after a failed run) and waits
        until every chunk has left.  After a failed run the chunks already
        queued still go first (rank 0 receives in order), and a failure of
        one of them does not keep the end marker back."""
        flag = CHUNK_ERROR if error else CHUNK_END
        first_exc = None
        for f in self.futs:
            try:
                f.result()
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                if first_exc is None:
                    first_exc = e
                flag = CHUNK_ERROR
        self.futs = []
        try:
            self.pool.submit(self._send, np.zeros(1, np.int64), np.zeros(0, np.uint8), flag).result()
        finally:
            self.pool.shutdown()
        if first_exc is not None and not error:
            raise first_exc


class ChunkReceiver:
    """rank 0 of a chunked step: one receive thread per peer takes that
    peer's chunks as they arrive (each into buffers of its own) while rank 0
    computes its own rows, so a slow peer holds back only its own chunks
    (on nccl each peer's point-to-point traffic runs on its own pair
    communicator and stream).  The threads are daemons: a rank-0 failure
    never leaves the interpreter waiting on them at exit."""

    def __init__(self, world, device=None):
        import threading
        import time
        self.world = world
        self.device = device
        self.per = {r: [] for r in range(1, world)}
        self.arrival = {r: [] for r in range(1, world)}  # perf_counter of each chunk's arrival
        self.status = {r: None for r in range(1, world)}  # "end", "error", or an exception
        self._t0 = time.perf_counter
        self.threads = [threading.Thread(target=self._peer, args=(r,), daemon=True,
                                         name=f"chunk-recv-{r}") for r in range(1, world)]
        for t in self.threads:
            t.start()

    def _peer(self, r):
        import torch
        import torch.distributed as dist
        try:
            dev = self.device if self.device is not None else torch.device("cpu")
            on_gpu = dev.type != "cpu"
            if on_gpu:
                torch.cuda.set_device(dev)
            while True:
                hdr = torch.empty(3, dtype=torch.int64, device=dev)
                for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, hdr, r)]):
                    w.wait()
                no, nd, flag = (int(x) for x in hdr.cpu())
                if flag == CHUNK_END:
                    self.status[r] = "end"
                    return
                if flag == CHUNK_ERROR:
                    self.status[r] = "error"
                    return
                flat = torch.empty(no + nd, dtype=torch.uint8, device=dev)
                ops = []
                if no:
                    ops.append(dist.P2POp(dist.irecv, flat[:no], r))
                if nd:
                    ops.append(dist.P2POp(dist.irecv, flat[no:], r))
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
                host = (flat.cpu() if on_gpu else flat).numpy()
                self.per[r].append((host[:no].view(np.int64), host[no:]))
                self.arrival[r].append(self._t0())
        except BaseException as e:  # noqa: BLE001 -- reported by result()
            self.status[r] = e

    def result(self, timeout=None):
        """Every peer's chunks in order ({rank: [(offsets, data), ...]});
        raises if a peer reported a failed run or a receive failed, and
        TimeoutError if a peer has not finished within `timeout` seconds."""
        import time
        deadline = None if timeout is None else time.monotonic() + timeout
        for t in self.threads:
            t.join(None if deadline is None else max(0.0, deadline - time.monotonic()))
            if t.is_alive():
                raise TimeoutError(f"{t.name}: peer still sending after {timeout} s")
        failed = {r: s for r, s in self.status.items() if s != "end"}
        if failed:
            r, s = sorted(failed.items())[0]
            if s == "error":
                raise RuntimeError(f"rank {r} reported a failed run (chunked gather)")
            raise RuntimeError(f"chunked gather: receiving from rank {r} failed: {s!r}") from (
                s if isinstance(s, BaseException) else None)
        return self.per


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
        self.gatherer = None
        self.tail_ms = []  # step_chunked: per step, the gather time left after the compute
        self.last_arrival = None  # step_chunked, rank 0: per peer, the arrival time of each chunk
        self.drain_timeout_s = 120.0  # step_chunked, rank 0 after its own failure

    @property
    def local_rows(self) -> tuple[int, int]:
        """The rank's output rows as indices into its loaded table slice."""
        return self.row_begin - self.table_begin, self.row_end - self.table_begin

    def pairs(self) -> int:
        return int(pairs_per_row(self.total_images, self.overlap)[self.row_begin:self.row_end].sum())

    def step(self, runner, device=None, background: bool = False, keep: bool = True):
        """One pass of the op over this rank's rows: `runner.table_run_packed`
        (the scm_table_run_packed binding, or a stand-in with the same
        result shape), then for world > 1 the gather of the packed io.cc rows
        to rank 0.  Returns (this rank's packed rows, the gathered per-rank
        (offsets, data) on rank 0 / None).  With `background` the gather runs
        on the plan's Gatherer thread while the caller goes on (the next
        step's compute), the second value is None, and drain() returns the
        gathered results (`keep` False: the result is dropped once done, as
        the bench does)."""
        lb, le = self.local_rows
        packed = runner.table_run_packed(self.overlap, lb, le)
        gathered = None
        if self.world > 1:
            if background:
                if self.gatherer is None:
                    self.gatherer = Gatherer(device)
                self.gatherer.submit(packed, keep)
            else:
                gathered = gather_packed(packed.offsets, packed.data, device)
        return packed, gathered

    def step_chunked(self, runner, device=None):
        """One pass over this rank's rows with the gather inside the step:
        `runner.table_run_chunks` (scm_table_run_chunks) hands over each
        batch's rows as soon as they are serialised and they travel to rank 0
        while the next batches compute, so only the last batch's rows are
        exposed after the compute.  Returns on rank 0 the gathered (offsets,
        data) chunks of every rank in row order (merge_gathered's input),
        elsewhere None.  World 1: the rank's own chunks."""
        lb, le = self.local_rows
        own = []
        if self.world == 1:
            runner.table_run_chunks(self.overlap, lb, le,
                                    lambda first, pk: own.append((pk.offsets, pk.data)))
            return own
        import time
        if self.rank == 0:
            recv = ChunkReceiver(self.world, device)
            try:
                runner.table_run_chunks(self.overlap, lb, le,
                                        lambda first, pk: own.append((pk.offsets, pk.data)))
            except BaseException:
                # The peers still send their rows and end markers; take them
                # (bounded) so that the job ends cleanly, then fail.
                try:
                    recv.result(timeout=self.drain_timeout_s)
                except Exception:  # noqa: BLE001 -- rank 0's own failure is the one raised
                    pass
                raise
            t0 = time.perf_counter()
            per = recv.result()
            self.tail_ms.append((time.perf_counter() - t0) * 1e3)
            self.last_arrival = recv.arrival
            return own + [c for r in range(1, self.world) for c in per[r]]
        snd = ChunkSender(device)
        try:
            runner.table_run_chunks(self.overlap, lb, le, lambda first, pk: snd.submit(pk))
        except BaseException:
            snd.finish(error=True)  # rank 0 raises instead of waiting for this rank's rows
            raise
        t0 = time.perf_counter()
        snd.finish()
        self.tail_ms.append((time.perf_counter() - t0) * 1e3)
        return None

    def run_passes(self, runner, passes: int, device=None, keep: bool = True):
        """`passes` steps as one streamed run (`runner.table_run_passes`, the
        scm_table_run_passes binding: the batches of step k + 1 enter the GPU
        pipeline while step k's last batches are verified).  For world > 1 each
        step's packed rows go to the plan's Gatherer as soon as the library
        hands them over, so the gather of step k overlaps the compute of the
        steps after it; drain() returns the gathered results.  Returns the last
        step's packed rows."""
        lb, le = self.local_rows
        last = {}

        def on_pass(k, packed):
            last["packed"] = packed
            if self.world > 1:
                if self.gatherer is None:
                    self.gatherer = Gatherer(device)
                self.gatherer.submit(packed, keep)

        runner.table_run_passes(self.overlap, lb, le, passes, on_pass)
        return last.get("packed")

    def drain(self) -> list:
        """Wait for the background gathers; rank 0: their results in step order."""
        return self.gatherer.drain() if self.gatherer is not None else []


def merge_gathered(payloads: list) -> tuple[list[bytes], list[bytes]]:
    """Rank 0: concatenate the gathered per-rank packed rows (gather_packed's
    (offsets, data) pairs) in rank order (= pivot-row order) into
    (pair_image_ids rows, two_view_geometries rows)."""
    rows_a, rows_b = [], []
    for offs, data in payloads:
        for r in range((len(offs) - 1) // 2):
            rows_a.append(data[offs[2 * r]:offs[2 * r + 1]].tobytes())
            rows_b.append(data[offs[2 * r + 1]:offs[2 * r + 2]].tobytes())
    return rows_a, rows_b
