"""Batch pipeline of the table path: packed output, kept matches, several
batches in flight (SCM_BATCH_PAIRS forces small batches), ragged tables.
Every output byte is compared with the CPU oracle (oracle/oracle.cc)."""
import os

import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd import Context
from scanner_colmap_amd.codecs import (decode_descriptors, decode_keypoints, encode_descriptors,
                                       encode_keypoints, table_rows)
from scanner_colmap_amd.synthetic import Corridor

pytestmark = pytest.mark.gpu


def _table(n, kpts, seed, overlap=4):
    imgs = Corridor(n, kpts, overlap, seed=seed).images()
    return imgs, table_rows(imgs)


def test_packed_equals_rows_and_oracle(gpu_ctx):
    imgs, (ids, kps, descs) = _table(9, 600, 31)
    ref = oracle.table_run(ids, kps, descs, 5, 0, len(imgs))
    gpu_ctx.table_load(ids, kps, descs)
    packed = gpu_ctx.table_run_packed(5, 0, len(imgs))
    pa, pb = packed.rows()
    assert pa == ref[0] and pb == ref[1]
    assert packed.offsets[-1] == packed.data.size
    rows = gpu_ctx.table_run(5, 0, len(imgs))
    assert rows[0] == pa and rows[1] == pb


def test_sub_range(gpu_ctx):
    imgs, (ids, kps, descs) = _table(8, 500, 37)
    ref = oracle.table_run(ids, kps, descs, 3, 2, 7)
    gpu_ctx.table_load(ids, kps, descs)
    got = gpu_ctx.table_run(3, 2, 7)
    assert got == ref
    empty = gpu_ctx.table_run_packed(3, 4, 4)
    assert len(empty) == 0 and empty.data.size == 0


def test_keep_matches(gpu_ctx):
    imgs, (ids, kps, descs) = _table(5, 800, 41)
    gpu_ctx.table_load(ids, kps, descs)
    gpu_ctx.set_keep_matches(True)
    try:
        gpu_ctx.table_run(3, 0, len(imgs))
        for r in range(len(imgs) - 1):
            for off in (1, 2):
                if r + off >= len(imgs):
                    continue
                got = gpu_ctx.table_matches(r, off)
                ref = oracle.match_pair(imgs[r][2], imgs[r + off][2])
                assert got.shape == ref.shape and (got == ref).all(), (r, off)
    finally:
        gpu_ctx.set_keep_matches(False)


@pytest.mark.parametrize("env", [{"SCM_BATCH_PAIRS": "3"},
                                 {"SCM_BATCH_PAIRS": "3", "SCM_SERIAL": "1"},
                                 {"SCM_BATCH_BYTES": str(6 << 20)}])
def test_many_batches_in_flight(env):
    """Batches of 3 pairs (or cut by a 6 MiB workspace budget, ~4 pairs of
    these images, scm_runtime.cpp set_budget_bytes): exercises the three
    rotating batch sets, the enqueue / collect alternation, the serial
    diagnostic schedule and per-batch serialisation against the oracle."""
    imgs, (ids, kps, descs) = _table(12, 400, 43)
    ref = oracle.table_run(ids, kps, descs, 4, 0, len(imgs))
    os.environ.update(env)
    try:
        with Context(0) as ctx:
            ctx.table_load(ids, kps, descs)
            got = ctx.table_run(4, 0, len(imgs))
            got2 = ctx.table_run_packed(4, 0, len(imgs)).rows()
            launches = ctx.table_timings()["match_launches"]
    finally:
        for k in env:
            del os.environ[k]
    assert got == ref
    assert got2 == ref
    assert launches >= 4  # the budget or the pair cap cut the table into several batches


def test_ragged_table_with_empty_images(gpu_ctx):
    """Images with 0, 1, 31 and 2000 keypoints in one table."""
    sizes = [700, 0, 1, 700, 31, 2000, 650]
    _, (ids, kps, descs) = _table(len(sizes), 2000, 47)
    kps2 = [encode_keypoints(decode_keypoints(k)[:s]) for s, k in zip(sizes, kps)]
    descs2 = [encode_descriptors(decode_descriptors(d)[:s]) for s, d in zip(sizes, descs)]
    ref = oracle.table_run(ids, kps2, descs2, 4, 0, len(sizes))
    gpu_ctx.table_load(ids, kps2, descs2)
    got = gpu_ctx.table_run(4, 0, len(sizes))
    assert got == ref


@pytest.mark.parametrize("batch_pairs", [None, "7"])
def test_streamed_passes_equal_single_runs(batch_pairs):
    """scm_table_run_passes: three passes of a row range as one batch stream
    (with 7-pair batches a batch spans every pass boundary): each pass's
    packed rows are byte-equal to the CPU oracle's table run, passes arrive in
    order, and the kept matches are the last pass's."""
    imgs, (ids, kps, descs) = _table(11, 500, 43)
    ref = oracle.table_run(ids, kps, descs, 4, 1, 10)
    if batch_pairs:
        os.environ["SCM_BATCH_PAIRS"] = batch_pairs
    try:
        with Context(0) as ctx:
            ctx.table_load(ids, kps, descs)
            ctx.set_keep_matches(True)
            got = []
            ctx.table_run_passes(4, 1, 10, 3, lambda k, p: got.append((k, p.rows())))
            assert [k for k, _ in got] == [0, 1, 2]
            for _, (pa, pb) in got:
                assert pa == ref[0] and pb == ref[1]
            m = ctx.table_matches(3, 2)
            r = oracle.match_pair(imgs[3][2], imgs[5][2])
            assert m.shape == r.shape and (m == r).all()
            ctx.set_keep_matches(False)
            empty = []
            ctx.table_run_passes(4, 5, 5, 2, lambda k, p: empty.append(len(p)))
            assert empty == [0, 0]
    finally:
        os.environ.pop("SCM_BATCH_PAIRS", None)


@pytest.mark.parametrize("batch_pairs", ["7", None])
def test_chunks_concatenate_to_packed(batch_pairs):
    """scm_table_run_chunks hands the rows over batch by batch (several
    batches with 7-pair batches, one without): the chunks cover the row range
    in order and their rows are scm_table_run_packed's / the oracle's; an
    empty range hands over nothing."""
    imgs, (ids, kps, descs) = _table(12, 500, 43)
    ref = oracle.table_run(ids, kps, descs, 4, 1, 11)
    if batch_pairs:
        os.environ["SCM_BATCH_PAIRS"] = batch_pairs
    try:
        with Context(0) as ctx:
            ctx.table_load(ids, kps, descs)
            chunks = []
            ctx.table_run_chunks(4, 1, 11, lambda first, pk: chunks.append((first, pk)))
            empty = []
            ctx.table_run_chunks(4, 5, 5, lambda first, pk: empty.append(first))
    finally:
        os.environ.pop("SCM_BATCH_PAIRS", None)
    assert empty == []
    assert (len(chunks) > 1) == (batch_pairs is not None)
    row = 1
    rows_a, rows_b = [], []
    for first, pk in chunks:
        assert first == row
        a, b = pk.rows()
        rows_a += a
        rows_b += b
        row += len(pk)
    assert row == 11
    assert (rows_a, rows_b) == ref
