"""GPU parity at the BASELINE.json sizes, through the C
ABI: 8192 x 8192-keypoint pairs (16 row blocks: the finalize kernel's 4-way
column merge, the XCD job order, full 8192-column segments), the Gerrard Hall
shape (100 images, overlap 10), a prefix of the 1000 x 8192 overlap-20 roofline
workload, the South-Building shape (exhaustive) and the 10000 x 4096 overlap-50
shape (prefix, several batches in flight).

The oracle's matcher here is oracle.match_pair_fast: the exact integer dot
matrix from a float32 BLAS product (every partial sum an integer < 2^24) fed to
the oracle's own FindBestMatches scans; tests/test_oracle_match.py pins it to
the faithful scalar matcher.  Keypoint counts below 8192 are reductions of the
real datasets' sizes chosen so the oracle finishes in seconds; the synthetic
scenes are the bench's generator (no dataset is available).  Images are
generated in-process (no forked workers once the GPU runtime is up)."""
import os

import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd import Context
from scanner_colmap_amd.codecs import decode_tvg, decode_tvg_list, table_rows
from scanner_colmap_amd.synthetic import Corridor

pytestmark = pytest.mark.gpu
THREADS = 16


def _check_table(ctx, imgs, overlap, rows=None):
    rows = rows or (0, len(imgs))
    ids, kps, descs = table_rows(imgs)
    ref_m = {}
    ref = oracle.table_run_fast(imgs, overlap, rows[0], rows[1], threads=THREADS,
                                matches_out=ref_m)
    ctx.table_load(ids, kps, descs)
    ctx.set_keep_matches(True)
    try:
        got = ctx.table_run(overlap, rows[0], rows[1])
        for (r, s), m in ref_m.items():
            g = ctx.table_matches(r, s - r, cap=max(1, len(m) + 1))
            assert g.shape == m.shape and (g == m).all(), (r, s)
    finally:
        ctx.set_keep_matches(False)
    assert got[0] == ref[0]
    for i, (a, b) in enumerate(zip(got[1], ref[1])):
        assert a == b, i
    configs = [t.config for row in got[1] for t in decode_tvg_list(row)]
    return configs


def test_pair_8192_bit_exact(gpu_ctx):
    """Config 3's pair shape: 8192 x 8192 (n1 > 2048 -> 16 row blocks)."""
    c = Corridor(20, 8192, 20, seed=20252)
    im = {i: c.image(i) for i in (0, 1, 10, 19)}
    for j in (1, 10, 19):
        got = gpu_ctx.match_pair(im[0][2], im[j][2])
        ref = oracle.match_pair_fast(im[0][2], im[j][2])
        assert got.shape == ref.shape and (got == ref).all(), j
        assert len(ref) > 100
        tg = gpu_ctx.verify_pair(im[0][1], im[j][1], ref, im[0][0], im[j][0])
        tr = oracle.verify_pair(im[0][1], im[j][1], ref, im[0][0], im[j][0])
        assert tg == tr, j
        assert decode_tvg(tr).config in (3, 6)


def test_pair_8192_ragged_and_reversed(gpu_ctx):
    """Ragged full-size pairs: 8192 x 5000 and 5000 x 8192 (partial last
    row block / column tile), and the same image against itself (every row a
    tie with its own column)."""
    c = Corridor(3, 8192, 3, seed=77)
    a, b = c.image(0)[2], c.image(1)[2][:5000]
    for x, y in ((a, b), (b, a), (a, a)):
        got = gpu_ctx.match_pair(x, y)
        ref = oracle.match_pair_fast(x, y)
        assert got.shape == ref.shape and (got == ref).all()


def test_gerrard_hall_shape_table():
    """Configs 1/2 at the metric's size: 100 images x 8192 keypoints, overlap
    10 (855 pairs, the bench's gerrard-hall-synth workload), every output row
    and every pair's raw matches bit-identical to the CPU op's."""
    imgs = Corridor(100, 8192, 10, seed=20251).images()
    with Context(0) as ctx:
        configs = _check_table(ctx, imgs, 10)
    assert len(configs) == 855


def test_roofline_workload_prefix():
    """Config 3 (1000 x 8192, overlap 20): its first 24 images at full size
    (266 pairs)."""
    imgs = Corridor(1000, 8192, 20, seed=20252).images(0, 24)
    with Context(0) as ctx:
        configs = _check_table(ctx, imgs, 20)
    assert len(configs) == 266


def test_exhaustive_shape():
    """Config 4 shape (South-Building exhaustive: overlap = number of images):
    48 images x 2048 (1,128 pairs: one batch above the small-batch threshold,
    verify_small_batch_pairs, so the table path's window kernels)."""
    imgs = Corridor(48, 2048, 48, seed=20253).images()
    with Context(0) as ctx:
        configs = _check_table(ctx, imgs, 48)
    assert len(configs) == 1128


def test_exhaustive_full_size_config4():
    """Config 4 at its own size: the bench's south-building-synth workload
    (128 images x 8192 keypoints, exhaustive: stencil range(0, 128), every
    one of the 8,128 pairs on one GPU through the HIP table path).
    Every row's pair ids follow the stencil rule of
    sequential_matching.cc:139-146 (feature_matching.py:43 with K = N); a
    fixed sample of pairs -- pivot row 0's first and last 8 neighbours, all
    of row 63, rows 120-126 -- has raw matches bit-exact and TwoViewGeometry
    bytes equal to the CPU oracle's."""
    from scanner_colmap_amd.codecs import decode_pair_ids, split_tvg_list
    n, k = 128, 8192
    imgs = Corridor(n, k, n, seed=20253).images()
    ids, kps, descs = table_rows(imgs)
    sample = {0: list(range(1, 9)) + list(range(120, 128)), 63: list(range(64, 128))}
    for r in range(120, 127):
        sample[r] = list(range(r + 1, 128))
    with Context(0) as ctx:
        ctx.table_load(ids, kps, descs)
        for r in sample:
            ctx.add_keep_matches_range(r, r + 1)
        got_ids, got_tvg = ctx.table_run(n, 0, n)
        got_m = {(r, s): ctx.table_matches(r, s - r) for r in sample for s in sample[r]}
        ctx.set_keep_matches(False)
    assert len(got_ids) == n and len(got_tvg) == n
    for r in range(n):
        assert decode_pair_ids(got_ids[r]) == [imgs[s][0] for s in range(r + 1, n)], r
    assert sum(len(decode_pair_ids(b)) for b in got_ids) == n * (n - 1) // 2

    def one(job):
        r, s = job
        m = oracle.match_pair_fast(imgs[r][2], imgs[s][2])
        return m, oracle.verify_pair(imgs[r][1], imgs[s][1], m, imgs[r][0], imgs[s][0])

    from concurrent.futures import ThreadPoolExecutor
    jobs = [(r, s) for r in sample for s in sample[r]]
    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        ref = dict(zip(jobs, ex.map(one, jobs)))
    for r in sample:
        row = split_tvg_list(got_tvg[r])
        assert len(row) == n - 1 - r
        for s in sample[r]:
            m, tvg = ref[(r, s)]
            g = got_m[(r, s)]
            assert g.shape == m.shape and (g == m).all(), (r, s)
            assert row[s - r - 1] == tvg, (r, s)
    assert len(jobs) == 16 + 64 + 28


def test_k50_shape_many_batches():
    """Config 5 shape (4096 kpts, overlap 50): 64 images (1,911 pairs) in
    batches of 400 pairs, so several batches are in flight at once (each on
    the small-batch kernels, whose replay and early-final streams are the
    other sets' verification streams, here busy with their own batches)."""
    imgs = Corridor(10000, 4096, 50, seed=20254).images(0, 64)
    os.environ["SCM_BATCH_PAIRS"] = "400"
    try:
        with Context(0) as ctx:
            configs = _check_table(ctx, imgs, 50)
    finally:
        del os.environ["SCM_BATCH_PAIRS"]
    assert len(configs) == sum(min(49, 63 - i) for i in range(64))


def test_config5_full_table_rank_share():
    """Config 5 at its size on one GPU: the whole 10,000 x 4096-keypoint table
    (overlap 50, 488,775 pairs, 5.2 GB of descriptors) resident in HBM, and one
    strong-scaled rank's share of the 8-GPU job (ShardPlan(10000, 50, 8, 3,
    "strong"): ~61K pairs) run through scm_table_run_packed.  Every row's pair
    ids follow the stencil rule (feature_matching.py:43,
    sequential_matching.cc:139-146); the rank's first row, a middle row and
    its last 4 rows have raw matches bit-exact and TwoViewGeometry bytes equal
    to the CPU oracle's; the packed byte volume the RCCL gather would ship is
    printed."""
    import time
    from concurrent.futures import ThreadPoolExecutor

    from scanner_colmap_amd.codecs import decode_pair_ids, split_tvg_list
    from scanner_colmap_amd.distributed import ShardPlan, pairs_per_row
    n, k, K = 10000, 4096, 50
    plan = ShardPlan(n, K, 8, 3, "strong")
    a, b = plan.row_begin, plan.row_end
    c = Corridor(n, k, K, seed=20255)
    t0 = time.perf_counter()
    ids, kps, descs = c.table_rows_spawned(0, n, workers=THREADS)
    t_gen = time.perf_counter() - t0
    sample = [a, (a + b) // 2] + list(range(b - 4, b))
    with Context(0) as ctx:
        ctx.table_load(ids, kps, descs)
        del kps, descs
        for r in sample:
            ctx.add_keep_matches_range(r, r + 1)
        t0 = time.perf_counter()
        packed = ctx.table_run_packed(K, a, b)
        t_run = time.perf_counter() - t0
        got_m = {(r, s): ctx.table_matches(r, s - r) for r in sample
                 for s in range(r + 1, min(n, r + K))}
    npairs = int(pairs_per_row(n, K)[a:b].sum())
    assert npairs == plan.pairs() and npairs > 60000
    assert len(packed) == b - a
    for r in range(a, b):
        got = decode_pair_ids(packed.element(2 * (r - a)))
        assert got == [s + 1 for s in range(r + 1, min(n, r + K))], r
    volume = int(packed.data.nbytes + packed.offsets.nbytes)
    print(f"config 5 rank 3 of 8: rows [{a}, {b}), {npairs} pairs, gen {t_gen:.1f} s, "
          f"run {t_run:.2f} s ({npairs / t_run:.0f} pairs/s incl. host rows), "
          f"gather volume {volume / 1e6:.1f} MB ({volume / npairs:.0f} B per pair)")
    imgs = {i: c.image(i) for i in {i for r in sample for i in range(r, min(n, r + K))}}

    def one(job):
        r, s = job
        m = oracle.match_pair_fast(imgs[r][2], imgs[s][2])
        return m, oracle.verify_pair(imgs[r][1], imgs[s][1], m, imgs[r][0], imgs[s][0])

    jobs = list(got_m)
    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        ref = dict(zip(jobs, ex.map(one, jobs)))
    for r in sample:
        row = split_tvg_list(packed.element(2 * (r - a) + 1))
        for s in range(r + 1, min(n, r + K)):
            m, tvg = ref[(r, s)]
            g = got_m[(r, s)]
            assert g.shape == m.shape and (g == m).all(), (r, s)
            assert row[s - r - 1] == tvg, (r, s)
    assert len(jobs) == 6 * (K - 1)
