"""GPU parity of kernel 1 (descriptor matching) against the CPU oracle:
match indices must be bit-exact (BASELINE north star).
Sizes are chosen so the oracle's faithful scalar matcher finishes in seconds."""
import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd.synthetic import Corridor, random_descriptors, tie_stress_pair

pytestmark = pytest.mark.gpu


def _same(ctx, a, b):
    got = ctx.match_pair(a, b)
    ref = oracle.match_pair(a, b)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(got, ref)
    return len(ref)


def test_random_ragged(gpu_ctx):
    a = random_descriptors(700, 1)
    b = random_descriptors(901, 2)
    b[:300] = a[100:400]
    _same(gpu_ctx, a, b)


def test_corridor_pairs(gpu_ctx):
    c = Corridor(4, 1500, 3, seed=5)
    imgs = c.images()
    n = [_same(gpu_ctx, imgs[0][2], imgs[j][2]) for j in (1, 2, 3)]
    assert n[0] > 100


def test_tie_stress(gpu_ctx):
    a, b = tie_stress_pair(1000, 777, 3)
    _same(gpu_ctx, a, b)
    _same(gpu_ctx, b, a)


def test_clamp_variant_large_norms(gpu_ctx):
    # Non-normalised descriptors (|a||b| >= 2^19) take the CLAMP kernel.
    rng = np.random.default_rng(9)
    a = rng.integers(0, 256, size=(600, 128), dtype=np.uint8)
    b = rng.integers(0, 256, size=(650, 128), dtype=np.uint8)
    b[:200] = a[:200]
    a[10] = 255
    b[20] = 255
    _same(gpu_ctx, a, b)


@pytest.mark.parametrize("n1,n2", [(0, 10), (10, 0), (1, 1), (1, 33), (33, 1), (31, 65),
                                   (513, 47)])
def test_edge_sizes(gpu_ctx, n1, n2):
    a = random_descriptors(max(n1, 1), 11)[:n1]
    b = random_descriptors(max(n2, 1), 12)[:n2]
    if n1 and n2:
        k = min(n1, n2)
        b[:k // 2] = a[:k // 2]
    _same(gpu_ctx, a, b)


def test_zero_descriptors(gpu_ctx):
    a = np.zeros((64, 128), np.uint8)
    b = random_descriptors(64, 3)
    _same(gpu_ctx, a, b)
    _same(gpu_ctx, b, a)


def test_segmented_columns(gpu_ctx):
    # n2 > 8192 exercises the column segments of the row state.
    a = random_descriptors(300, 21)
    b = random_descriptors(8192 + 700, 22)
    b[8500:8800] = a
    b[100:200] = a[:100]
    _same(gpu_ctx, a, b)


@pytest.mark.parametrize("n", [33, 81, 260])
def test_segmented_columns_batches(n):
    """Batches of pairs with n2 > 8192 through the table path, kept matches of
    every row against the oracle's pair matcher: 259 pairs make 2,452 one-pair
    matcher jobs, enough to fill the CUs, so the matcher sweeps whole pairs and
    crosses its own 8192-column row segments; 80 and 32 pairs take the column
    split into 2 and 4 parts (one-pair jobs below 1,024), whose 8892-column
    pairs need more tiles than a part's power-of-two width allows -- 2
    segments of 128 tiles, 3 of 64.  (A single pair, as in
    test_segmented_columns, takes 8 parts.)"""
    from scanner_colmap_amd import Context
    from scanner_colmap_amd.codecs import table_rows
    rng = np.random.default_rng(31)
    descs = [random_descriptors(64 if i % 2 == 0 else 8192 + 700, 300 + i) for i in range(n)]
    for i in range(0, n - 1, 2):
        descs[i + 1][8500:8564] = descs[i]  # pivot i's matches in the second segment
        descs[i + 1][100:132] = descs[i][:32]  # and duplicates in the first (ties)
    imgs = [(i + 1, np.concatenate([rng.uniform(0, 1000, (len(d), 2)),
                                    np.zeros((len(d), 4))], 1).astype(np.float32), d)
            for i, d in enumerate(descs)]
    ids, kps, enc = table_rows(imgs)
    with Context(0) as ctx:
        ctx.table_load(ids, kps, enc)
        ctx.set_keep_matches(True)
        ctx.table_run(2, 0, n)
        got = [ctx.table_matches(r, 1) for r in range(n - 1)]
    for r in range(n - 1):
        ref = oracle.match_pair(descs[r], descs[r + 1])
        np.testing.assert_array_equal(got[r], ref, err_msg=f"row {r}")
    assert sum(len(g) for g in got[0::2]) >= 32 * (n // 2)  # the even rows: 32 unique copies each


def test_high_bytes_fast_variant(gpu_ctx):
    # Bytes >= 128 (outside the i8 range before the offset) with norms small
    # enough for the fast keys: exercises the a - 128 correction terms.
    rng = np.random.default_rng(12)
    a = np.zeros((500, 128), np.uint8)
    b = np.zeros((520, 128), np.uint8)
    for m in (a, b):
        idx = rng.integers(0, 128, size=(m.shape[0], 4))
        np.put_along_axis(m, idx, rng.integers(128, 256, size=(m.shape[0], 4)).astype(np.uint8), 1)
        m += rng.integers(0, 3, size=m.shape, dtype=np.uint8)
    b[:150] = a[50:200]
    _same(gpu_ctx, a, b)


def test_bf16_matcher_parity(monkeypatch):
    """SCM_MATCH_BF16=1 selects the bf16 MFMA matcher; it is bit-exact too."""
    from scanner_colmap_amd import Context
    monkeypatch.setenv("SCM_MATCH_BF16", "1")
    ctx = Context(0)
    try:
        a, b = tie_stress_pair(1000, 777, 3)
        _same(ctx, a, b)
        imgs = Corridor(3, 1500, 3, seed=6).images()
        _same(ctx, imgs[0][2], imgs[2][2])
        rng = np.random.default_rng(10)
        x = rng.integers(0, 256, size=(300, 128), dtype=np.uint8)
        y = rng.integers(0, 256, size=(333, 128), dtype=np.uint8)
        y[:100] = x[:100]
        _same(ctx, x, y)
    finally:
        ctx.close()


def _opts_pair(**kw):
    from scanner_colmap_amd import default_options
    o_gpu, o_ref = default_options(), oracle.default_options()
    for k, v in kw.items():
        setattr(o_gpu, k, v)
        setattr(o_ref, k, v)
    return o_gpu, o_ref


@pytest.mark.parametrize("kw", [dict(max_ratio=1.5, max_distance=3.0),
                                dict(cross_check=0),
                                dict(cross_check=0, max_ratio=1.2),
                                dict(max_ratio=1.0)])
def test_option_variants(kw):
    """max_ratio > 1 lets tied bests pass the ratio test, so the lowest-index
    tie rule decides the cross-check: the runtime switches to the bf16 matcher
    (column keys).  max_ratio <= 1 and cross_check off stay on the i8 matcher
    (column values).  All are bit-exact against the oracle."""
    from scanner_colmap_amd import Context
    o_gpu, o_ref = _opts_pair(**kw)
    ctx = Context(0, o_gpu)
    try:
        cases = [tie_stress_pair(1000, 777, 3), tie_stress_pair(600, 900, 4)]
        rng = np.random.default_rng(21)
        x = rng.integers(0, 256, size=(300, 128), dtype=np.uint8)
        y = rng.integers(0, 256, size=(333, 128), dtype=np.uint8)
        y[:100] = x[:100]
        y[100:150] = x[:50]  # duplicated columns: tied column bests
        cases.append((x, y))
        imgs = Corridor(3, 1200, 3, seed=8).images()
        cases.append((imgs[0][2], imgs[1][2]))
        for a, b in cases:
            got = ctx.match_pair(a, b)
            ref = oracle.match_pair(a, b, o_ref)
            np.testing.assert_array_equal(got, ref)
    finally:
        ctx.close()
