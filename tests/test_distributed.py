"""Multi-rank plumbing on the CPU: pair-balanced sharding
with halos, and the rank-0 gather of packed io.cc rows over a world-size-2
gloo group.  Each rank computes its shard with the CPU oracle standing in
for the GPU stage; rank 0 checks the gathered rows against a one-rank run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from scanner_colmap_amd import distributed as sd


@pytest.mark.parametrize("n,K,world", [(100, 10, 8), (1000, 20, 8), (128, 128, 8), (7, 4, 2),
                                       (3, 10, 4), (0, 5, 2)])
def test_shard_rows_partition(n, K, world):
    ppr = sd.pairs_per_row(n, K)
    bounds = [sd.shard_rows(n, K, world, r) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    for (a, b), (c, _) in zip(bounds, bounds[1:]):
        assert b == c and a <= b
    loads = [int(ppr[a:b].sum()) for a, b in bounds]
    if n > 0 and ppr.sum() > 0:
        assert max(loads) - min(loads) <= max(ppr) + 1 or min(loads) == 0
        assert sum(loads) == ppr.sum()
    for a, b in bounds:
        ta, tb = sd.table_range(a, b, n, K)
        assert ta == a and tb == min(n, b + K - 1)


def test_merge_gathered():
    """Rank 0's per-rank (offsets, packed bytes) payloads -> the two output
    columns' rows in rank order; empty ranks contribute nothing."""
    rows_a = [b"\x01\x00\x00\x00\x00\x00\x00\x00\x05\x00\x00\x00", b"\x00" * 8]
    rows_b = [b"abc" * 5, b"\x0c" + b"\x00" * 11]
    data = b"".join(x for pair in zip(rows_a, rows_b) for x in pair)
    offs = np.cumsum([0] + [len(x) for pair in zip(rows_a, rows_b) for x in pair]).astype(np.int64)
    empty = (np.zeros(1, np.int64), np.zeros(0, np.uint8))
    got = sd.merge_gathered([(offs[:3], np.frombuffer(data, np.uint8)[:offs[2]]), empty,
                             (offs[2:] - offs[2], np.frombuffer(data, np.uint8)[offs[2]:])])
    assert got == (rows_a, rows_b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _OracleRunner:
    """Stand-in for the GPU context in the CPU test: the same
    table_run_packed result shape (offsets + packed element bytes), computed
    by the CPU oracle over the rank's loaded table slice."""

    def __init__(self, ids, kps, descs):
        self.table = (ids, kps, descs)

    def table_run_packed(self, overlap, row_begin, row_end):
        from oracle import oracle
        pa, pb = oracle.table_run(*self.table, overlap, row_begin, row_end)
        elems = [x for pair in zip(pa, pb) for x in pair]

        class _P:
            offsets = np.cumsum([0] + [len(x) for x in elems]).astype(np.int64)
            data = (np.frombuffer(b"".join(elems), np.uint8) if elems
                    else np.zeros(0, np.uint8))
        return _P()

    def table_run_chunks(self, overlap, row_begin, row_end, on_chunk, rows_per_chunk=2):
        # scm_table_run_chunks' contract: the rows in order, a batch of rows at a time
        for a in range(row_begin, row_end, rows_per_chunk):
            on_chunk(a, self.table_run_packed(overlap, a, min(row_end, a + rows_per_chunk)))

    def table_run_passes(self, overlap, row_begin, row_end, passes, on_pass):
        # scm_table_run_passes' contract: each pass's packed rows, in order
        for k in range(passes):
            on_pass(k, self.table_run_packed(overlap, row_begin, row_end))


def _rank_main(rank, world, port, n, K, scaling, q, background=False, steps=1, streamed=False,
               chunked=False):
    import torch.distributed as dist

    from oracle import oracle
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # bench.py's own sharding and step: ShardPlan -> table slice with the
        # halo -> runner.table_run_packed over the local rows -> P2P gather
        # (synchronous, or on the plan's background thread over several steps)
        plan = sd.ShardPlan(n, K, world, rank, scaling)
        c = Corridor(plan.total_images, 400, K, seed=53)
        runner = _OracleRunner(*table_rows(c.images(plan.table_begin, plan.table_end)))
        results = []
        if chunked:  # the gather inside the step, batch by batch
            results = [plan.step_chunked(runner) for _ in range(steps)]
            if rank != 0:
                assert results == [None] * steps
                results = []
        elif streamed:  # the steps as one streamed run
            last = plan.run_passes(runner, steps)
            assert last is not None
            results = [None] * steps
        else:
            for _ in range(steps):
                _, got = plan.step(runner, background=background)
                results.append(got)
        if (background or streamed) and not chunked:
            assert results == [None] * steps
            results = plan.drain()
        if rank == 0:
            ids, kps, descs = table_rows(c.images())
            ref = oracle.table_run(ids, kps, descs, K, 0, plan.total_images)
            ok = [sd.merge_gathered(g) == (ref[0], ref[1]) for g in results]
            rows_a, _ = sd.merge_gathered(results[-1])
            q.put((all(ok) and len(ok) == steps, True, len(rows_a), plan.total_images))
        else:
            assert all(g is None for g in results)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,K,scaling", [(9, 4, "strong"), (5, 3, "weak"), (2, 5, "strong")])
def test_gloo_shard_step_world2(n, K, scaling):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, K, scaling, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    assert codes == [0, 0], codes
    ok_a, ok_b, nrows, total = q.get(timeout=5)
    assert ok_a and ok_b and nrows == total
    assert total == (n if scaling == "strong" else n * world)


def _payload(rank, n):
    rng = np.random.default_rng(rank)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    cuts = np.sort(rng.integers(0, n + 1, 4)) if n else np.zeros(4, np.int64)
    return np.concatenate([[0], cuts, [n]]).astype(np.int64), data


def _gather_main(rank, world, port, sizes, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        offs, data = _payload(rank, sizes[rank])
        got = sd.gather_packed(offs, data)
        if rank == 0:
            ok = len(got) == world
            for r in range(world):
                ro, rd = _payload(r, sizes[r])
                ok = ok and (got[r][0] == ro).all() and got[r][1].tobytes() == rd.tobytes()
            q.put(bool(ok))
        else:
            q.put(got is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [[5, 0, 70000, 1], [0, 0, 0, 0], [0, 3, 0, 12345]])
def test_gloo_gather_world4_uneven_and_empty(sizes):
    """gather_packed (one batch_isend_irecv group, offsets and bytes as two
    messages per rank) at world 4: empty payloads on any rank (rank 0
    included), uneven sizes."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_main, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert [p.exitcode for p in procs] == [0] * world
    assert all(q.get(timeout=5) for _ in range(world))


def test_gloo_background_gather_world2():
    """The bench's overlapped form: three steps whose gathers run on the
    plan's background thread while the next step computes; drain() returns
    every step's gathered rows, each equal to a one-rank run."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, 7, 4, "strong", q, True, 3))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert [p.exitcode for p in procs] == [0, 0]
    ok, _, nrows, total = q.get(timeout=5)
    assert ok and nrows == total == 7


@pytest.mark.parametrize("n,K,scaling", [(6, 4, "strong"), (3, 5, "weak")])
def test_gloo_shard_step_world4(n, K, scaling):
    """ShardPlan.step at world 4: with 6 images strong-scaled some ranks own one
    row (or none with pairs), and the last rank's rows have no pairs at all."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, K, scaling, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert [p.exitcode for p in procs] == [0] * world
    ok_a, ok_b, nrows, total = q.get(timeout=5)
    assert ok_a and ok_b and nrows == total


def test_shard_plan_scaling():
    weak = [sd.ShardPlan(1000, 20, 8, r, "weak") for r in range(8)]
    strong = [sd.ShardPlan(10000, 50, 8, r, "strong") for r in range(8)]
    assert weak[0].total_images == 8000 and strong[0].total_images == 10000
    assert sum(p.pairs() for p in strong) == 488775  # BASELINE config 5
    assert sum(p.pairs() for p in [sd.ShardPlan(128, 128, 8, r, "strong") for r in range(8)]) == 8128
    with pytest.raises(ValueError):
        sd.ShardPlan(10, 3, 2, 0, "both")


def test_gloo_streamed_passes_world2():
    """ShardPlan.run_passes (bench.py's timed form): three steps as one
    streamed run, each step's rows handed to the gather thread as the runner
    produces them; drain() returns every step's rows, equal to a one-rank run."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main,
                         args=(r, world, port, 7, 4, "strong", q, False, 3, True))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert [p.exitcode for p in procs] == [0, 0]
    ok, _, nrows, total = q.get(timeout=5)
    assert ok and nrows == total == 7


@pytest.mark.parametrize("world,n,K,scaling", [(2, 9, 4, "strong"), (4, 6, 4, "strong"),
                                               (4, 3, 5, "weak"), (2, 2, 5, "strong")])
def test_gloo_chunked_step(world, n, K, scaling):
    """ShardPlan.step_chunked (the gather inside the step): every rank's rows
    leave batch by batch while the next batches compute; rank 0 receives each
    peer's chunks on a thread of its own, and the merged rows of two steps equal a
    one-rank run -- uneven chunk counts per rank, ranks without rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main,
                         args=(r, world, port, n, K, scaling, q, False, 2, False, True))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert [p.exitcode for p in procs] == [0] * world
    ok, _, nrows, total = q.get(timeout=5)
    assert ok and nrows == total


class _SyntheticChunks:
    """Stand-in runner for the chunked-gather tests: `nchunks` chunks of
    deterministic packed rows per rank; `sleep_after` = (chunk, seconds)
    pauses mid-step after that chunk, `fail_after` raises after that chunk."""

    def __init__(self, rank, nchunks, sleep_after=None, fail_after=None):
        self.rank, self.nchunks = rank, nchunks
        self.sleep_after, self.fail_after = sleep_after, fail_after

    @staticmethod
    def chunk(rank, k):
        offs, data = _payload(100 * rank + k, 1000 + 37 * k)
        return offs, data

    def table_run_chunks(self, overlap, row_begin, row_end, on_chunk):
        import time

        for k in range(self.nchunks):
            offs, data = self.chunk(self.rank, k)

            class _P:
                pass
            pk = _P()
            pk.offsets, pk.data = offs, data
            on_chunk(k, pk)
            if self.fail_after == k:
                raise RuntimeError(f"rank {self.rank}: runner failed after chunk {k}")
            if self.sleep_after and self.sleep_after[0] == k:
                time.sleep(self.sleep_after[1])


def _chunk_main(rank, world, port, q, sleepy=None, failing=None):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = sd.ShardPlan(8 * world, 3, world, rank, "strong")
        runner = _SyntheticChunks(rank, 3, sleep_after=(0, 3.0) if rank == sleepy else None,
                                  fail_after=0 if rank == failing else None)
        try:
            got = plan.step_chunked(runner)
        except Exception as e:  # noqa: BLE001 -- reported to the test
            q.put((rank, "raised", str(e)))
            return
        if rank == 0:
            want = [_SyntheticChunks.chunk(r, k) for r in range(world) for k in range(3)]
            same = len(got) == len(want) and all(
                (a[0] == b[0]).all() and a[1].tobytes() == b[1].tobytes() for a, b in zip(got, want))
            arr = plan.last_arrival
            q.put((rank, "ok", (bool(same), {r: list(v) for r, v in arr.items()})))
        else:
            q.put((rank, "ok", None))
    finally:
        dist.destroy_process_group()


def _run_chunk_world(world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunk_main, args=(r, world, port, q), kwargs=kw)
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank hung"
    out = {}
    while len(out) < world:
        r, what, info = q.get(timeout=5)
        out[r] = (what, info)
    return [p.exitcode for p in procs], out


def test_gloo_chunked_slow_rank_does_not_block_others():
    """Rank 0 receives each peer's chunks on that peer's own thread: while
    rank 1 sleeps 3 s after its first chunk, ranks 2 and 3 deliver all their
    chunks (a round-robin receiver would have waited on rank 1's second
    chunk first); the rows arrive in order and byte-equal."""
    codes, out = _run_chunk_world(4, sleepy=1)
    assert codes == [0] * 4
    same, arr = out[0][1]
    assert same
    late = arr[1][1]  # rank 1's second chunk comes after its sleep
    assert late - arr[1][0] > 2.5
    for r in (2, 3):
        assert len(arr[r]) == 3 and max(arr[r]) < late - 1.0, (r, arr)


@pytest.mark.parametrize("failing", [2, 0])
def test_gloo_chunked_failure_is_reported(failing):
    """A runner that raises mid-step: on a peer, its end marker carries the
    error flag and rank 0 raises naming it instead of waiting for rows that
    never come; on rank 0, the peers' chunks are still taken (the peers end
    cleanly) and rank 0 raises its own error.  No rank hangs."""
    world = 3
    codes, out = _run_chunk_world(world, failing=failing)
    assert codes == [0] * world  # every rank returned (the failures were reported, not hung)
    assert out[failing][0] == "raised" and "runner failed" in out[failing][1]
    if failing != 0:
        assert out[0][0] == "raised" and f"rank {failing} reported a failed run" in out[0][1]
    for r in range(world):
        if r not in (0, failing):
            assert out[r][0] == "ok"
