"""The N > 1 path with the real GPU stage: two ranks of
bench.py's own ShardPlan (pivot rows balanced by pair count, stencil halo),
each running scm_table_run_packed on a GPU context over its slice, the rows
gathered to rank 0 (gloo here: the ranks share the one GPU of the box, which
RCCL does not allow), compared with the oracle's whole-table rows.  The
CPU-only twin with the oracle as the stage is tests/test_distributed.py."""
import multiprocessing as mp
import os
import socket

import pytest

from scanner_colmap_amd import distributed as sd

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n, K, scaling, q, chunked=False, on_device=False):
    import torch
    import torch.distributed as dist

    from oracle import oracle
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = sd.ShardPlan(n, K, world, rank, scaling)
        c = Corridor(plan.total_images, 900, K, seed=57)
        if chunked:
            os.environ["SCM_BATCH_PAIRS"] = "5"  # several batches = several chunks per rank
        # on_device: the gather's device-staging branch (pinned staging, one
        # H2D hop, device messages, rank 0's D2H) -- the nccl path's, over gloo
        dev = torch.device("cuda:0") if on_device else None
        with Context(0) as ctx:
            ctx.table_load(*table_rows(c.images(plan.table_begin, plan.table_end)))
            if chunked:
                got = plan.step_chunked(ctx, dev)
                if rank == 0:
                    assert len(got) > world
            else:
                _, got = plan.step(ctx, dev)
        if rank == 0:
            rows_a, rows_b = sd.merge_gathered(got)
            ids, kps, descs = table_rows(c.images())
            ref = oracle.table_run(ids, kps, descs, K, 0, plan.total_images)
            q.put((rows_a == ref[0], rows_b == ref[1], len(rows_a), plan.total_images))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,K,scaling,chunked,on_device", [
    (11, 4, "strong", False, False), (6, 3, "weak", False, False), (11, 4, "strong", True, False),
    (11, 4, "strong", False, True), (11, 4, "strong", True, True)])
def test_gpu_shard_step_world2(n, K, scaling, chunked, on_device):
    """chunked: ShardPlan.step_chunked over scm_table_run_chunks (batches of 5
    pairs, so each rank hands over several chunks inside the step).
    on_device: the messages are device tensors staged as on nccl (RCCL itself
    refuses two ranks on one GPU, profiles/r05_rc_rccl_same_gpu.log)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, K, scaling, q, chunked, on_device))
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


def _rank_passes_main(rank, world, port, n, K, passes, q):
    import gc

    import torch.distributed as dist

    from oracle import oracle
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = sd.ShardPlan(n, K, world, rank, "strong")
        c = Corridor(plan.total_images, 800, K, seed=58)
        with Context(0) as ctx:
            ctx.table_load(*table_rows(c.images(plan.table_begin, plan.table_end)))
            plan.run_passes(ctx, passes, keep=True)
            gc.collect()
            # more library runs: their buffers come from the pool the kept
            # passes' PackedRows would have returned if the views did not hold them
            lb, le = plan.local_rows
            for _ in range(2):
                ctx.table_run_packed(K, lb, le)
            gathered = plan.drain()
        if rank == 0:
            ids, kps, descs = table_rows(c.images())
            ref = oracle.table_run(ids, kps, descs, K, 0, plan.total_images)
            q.put([sd.merge_gathered(g) == ref for g in gathered])
    finally:
        dist.destroy_process_group()


def test_gpu_streamed_passes_kept_world2():
    """ShardPlan.run_passes with keep=True over the real library
    (scm_table_run_passes): every pass's gathered rows stay byte-equal to the
    oracle after later passes and later runs, i.e. rank 0's own entry (a view
    of a library buffer) and the peers' entries outlive the buffer pool and
    the staging ring."""
    world, passes = 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_passes_main, args=(r, world, port, 12, 4, passes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert [p.exitcode for p in procs] == [0, 0]
    assert q.get(timeout=5) == [True] * passes
