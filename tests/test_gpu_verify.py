"""GPU parity of kernel 2 (two-view geometry: F / H LO-RANSAC, watermark,
post-filter) against the CPU oracle on identical seeded inputs: the io.cc TVG
bytes must be identical (config, F, H, inlier_matches)."""
import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd.codecs import decode_tvg, table_rows
from scanner_colmap_amd.synthetic import Corridor

pytestmark = pytest.mark.gpu


def test_verify_pairs_bytes(gpu_ctx):
    c = Corridor(5, 1200, 4, seed=13)
    imgs = c.images()
    for j in (1, 2, 3, 4):
        m = oracle.match_pair(imgs[0][2], imgs[j][2])
        ref = oracle.verify_pair(imgs[0][1], imgs[j][1], m, 1, j + 1)
        got = gpu_ctx.verify_pair(imgs[0][1], imgs[j][1], m, 1, j + 1)
        tr, tg = decode_tvg(ref), decode_tvg(got)
        assert tg.config == tr.config, (j, tg.config, tr.config)
        np.testing.assert_array_equal(tg.inlier_matches, tr.inlier_matches)
        np.testing.assert_array_equal(tg.F, tr.F)
        np.testing.assert_array_equal(tg.H, tr.H)
        assert got == ref


def test_verify_few_matches(gpu_ctx):
    c = Corridor(2, 200, 2, seed=3)
    imgs = c.images()
    m = oracle.match_pair(imgs[0][2], imgs[1][2])[:10]
    assert oracle.verify_pair(imgs[0][1], imgs[1][1], m, 1, 2) == \
        gpu_ctx.verify_pair(imgs[0][1], imgs[1][1], m, 1, 2)


def test_execute_stencil_bytes(gpu_ctx):
    c = Corridor(6, 900, 5, seed=17)
    imgs = c.images()
    ids, kps, descs = table_rows(imgs)
    ref = oracle.execute_stencil(ids, kps, descs)
    got = gpu_ctx.execute_stencil(ids, kps, descs)
    assert got[0] == ref[0]
    assert got[1] == ref[1]


def test_table_run_bytes(gpu_ctx):
    c = Corridor(10, 700, 4, seed=23)
    imgs = c.images()
    ids, kps, descs = table_rows(imgs)
    ref = oracle.table_run(ids, kps, descs, 4, 0, len(imgs))
    gpu_ctx.table_load(ids, kps, descs)
    got = gpu_ctx.table_run(4, 0, len(imgs))
    for i in range(len(imgs)):
        assert got[0][i] == ref[0][i], i
        assert got[1][i] == ref[1][i], i


@pytest.mark.parametrize("batch_pairs", ["0", "7"])
def test_profile_diagnostic_keeps_outputs(monkeypatch, capfd, batch_pairs):
    """SCM_PROFILE=1 (read at context creation) records per-pair phase cycles
    in the verification kernels and prints their summary at context
    destruction; the rows stay the oracle's.  With SCM_BATCH_PAIRS=7 the
    table runs as several batches (the pipelined form, the last batch among
    them)."""
    from scanner_colmap_amd import Context
    ids, kps, descs = table_rows(Corridor(10, 600, 4, seed=77).images())
    ref = oracle.table_run(ids, kps, descs, 4, 0, len(ids))
    monkeypatch.setenv("SCM_PROFILE", "1")
    if batch_pairs != "0":
        monkeypatch.setenv("SCM_BATCH_PAIRS", batch_pairs)
    with Context(0) as ctx:
        ctx.table_load(ids, kps, descs)
        assert ctx.table_run(4, 0, len(ids)) == ref
    assert "[scm verify profile]" in capfd.readouterr().err
