"""Every two-view-geometry outcome on the GPU, byte-equal to the CPU oracle
(reference sequential_matching.cc:84-101,
164-178): UNCALIBRATED, PLANAR_OR_PANORAMIC, WATERMARK, DEGENERATE with >= 15
matches (emptied by the post-filter), UNCALIBRATED with few inliers — through
scm_verify_pair against the committed fixtures and through the table path
(descriptors crafted so the matcher returns the scene's matches).  Also the
stencil dedup of execute() (repeated image ids, :139-146) and verification
option variants."""
import numpy as np
import pytest

from golden_util import OUTCOMES, load_outcomes
from oracle import oracle
from scanner_colmap_amd import Context, default_options
from scanner_colmap_amd.codecs import decode_tvg, decode_tvg_list, encode_image_id, table_rows
from scanner_colmap_amd.synthetic import (Corridor, descriptors_for_matches, geometry_scene)

pytestmark = pytest.mark.gpu
G = load_outcomes()


@pytest.mark.parametrize("name", sorted(OUTCOMES))
def test_verify_outcome_fixture(gpu_ctx, name):
    kp1, kp2, m, ids = (G[f"{name}_{k}"] for k in ("kp1", "kp2", "matches", "ids"))
    got = gpu_ctx.verify_pair(kp1, kp2, m, int(ids[0]), int(ids[1]))
    assert got == G[f"{name}_tvg"].tobytes()
    assert decode_tvg(got).config == OUTCOMES[name][1]


@pytest.mark.parametrize("kind,m,seed,expect", [("planar", 400, 11, 6), ("translation", 400, 12, 7),
                                                ("random", 45, 13, 0), ("general", 400, 14, 3)])
def test_table_path_outcomes(gpu_ctx, kind, m, seed, expect):
    kp1, kp2, mt = geometry_scene(kind, m, seed)
    d1, d2 = descriptors_for_matches(mt, m, m, seed)
    imgs = [(7, kp1, d1), (9, kp2, d2)]
    ids, kps, descs = table_rows(imgs)
    ref = oracle.table_run(ids, kps, descs, 2, 0, 2)
    gpu_ctx.table_load(ids, kps, descs)
    got = gpu_ctx.table_run(2, 0, 2)
    assert got == ref
    assert decode_tvg_list(got[1][0])[0].config == expect


def test_execute_stencil_repeated_ids(gpu_ctx):
    """Stencil ids [5, 6, 6, 5, 7, 6]: the pivot's own id and ids already
    paired are skipped (sequential_matching.cc:141-144) -> pairs (5, 6), (5, 7)."""
    imgs = Corridor(3, 700, 3, seed=19).images()
    by = {5: imgs[0], 6: imgs[1], 7: imgs[2]}
    order = [5, 6, 6, 5, 7, 6]
    ids = [encode_image_id(i) for i in order]
    _, kps, descs = table_rows([by[i] for i in order])
    ref = oracle.execute_stencil(ids, kps, descs)
    got = gpu_ctx.execute_stencil(ids, kps, descs)
    assert got == ref
    assert np.frombuffer(got[0], np.uint32, offset=8).tolist() == [6, 7]


@pytest.mark.parametrize("kw", [dict(detect_watermark=0), dict(min_num_inliers=40),
                                dict(max_error=2.0), dict(confidence=0.99, max_num_trials=500),
                                dict(max_H_inlier_ratio=0.95), dict(ransac_seed=12345),
                                dict(multiple_models=1),
                                dict(multiple_models=1, detect_watermark=0, ransac_seed=7)])
def test_verify_option_variants(kw):
    o_gpu, o_ref = default_options(), oracle.default_options()
    for k, v in kw.items():
        setattr(o_gpu, k, v)
        setattr(o_ref, k, v)
    with Context(0, o_gpu) as ctx:
        for kind, m, seed in (("translation", 300, 2), ("planar", 300, 1), ("general", 500, 3),
                              ("two_motions", 400, 21), ("general", 600, 22)):
            kp1, kp2, mt = geometry_scene(kind, m, seed)
            got = ctx.verify_pair(kp1, kp2, mt, 3, 4)
            assert got == oracle.verify_pair(kp1, kp2, mt, 3, 4, o_ref), (kw, kind)


def test_pair_with_more_than_65535_matches(gpu_ctx):
    # 32-bit sample indices: a pair of 70,000 matches (images of 70,000
    # keypoints) verifies like the oracle, through scm_verify_pair and through
    # the table path (the LDS-staged shuffle falls back to global memory)
    m = 70000
    kp1, kp2, mt = geometry_scene("general", m, 15)
    ref = oracle.verify_pair(kp1, kp2, mt, 3, 4)
    assert decode_tvg(ref).config == 3 and len(decode_tvg(ref).inlier_matches) > 50000
    assert gpu_ctx.verify_pair(kp1, kp2, mt, 3, 4) == ref
    d1, d2 = descriptors_for_matches(mt, m, m, 15)
    ids, kps, descs = table_rows([(3, kp1, d1), (4, kp2, d2)])
    gpu_ctx.table_load(ids, kps, descs)
    gpu_ctx.set_keep_matches(True)
    got_ids, got_tvg = gpu_ctx.table_run(2, 0, 2)
    got_m = gpu_ctx.table_matches(0, 1, cap=1 << 17)
    gpu_ctx.set_keep_matches(False)
    assert len(got_m) > 65535
    # descriptors_for_matches crafts descriptors whose matches are exactly mt
    # (oracle.match_pair_fast agrees at this size; a 20 GB dot matrix, not rerun here)
    assert got_m.shape == mt.shape and (got_m == mt).all()
    # the row's two_view_geometries element: size_t total, int count, then the TVG
    assert got_tvg[0][12:] == oracle.verify_pair(kp1, kp2, got_m, 3, 4)


@pytest.mark.parametrize("batch_pairs", [None, "3"])
def test_multiple_models_table_path(batch_pairs):
    """EstimateMultiple (multiple_models) through the table path: every pair
    of a batch runs its later Estimates together as given-match batches; rows
    byte-equal to the oracle's, including MULTIPLE (8) rows; small batches put
    several pipelined batches in flight."""
    import os
    scenes = [geometry_scene(k, m, s) for k, m, s in (("two_motions", 400, 21), ("general", 600, 22),
                                                       ("translation", 300, 2), ("planar", 300, 1),
                                                       ("two_motions", 300, 23))]
    imgs = []
    for i, (kp1, kp2, mt) in enumerate(scenes):
        d1, d2 = descriptors_for_matches(mt, len(kp1), len(kp2), 40 + i)
        imgs += [(100 + 2 * i, kp1, d1), (101 + 2 * i, kp2, d2)]
    ids, kps, descs = table_rows(imgs)
    o_gpu, o_ref = default_options(), oracle.default_options()
    o_gpu.multiple_models = o_ref.multiple_models = 1
    ref = oracle.table_run(ids, kps, descs, 2, 0, len(imgs), o_ref)
    if batch_pairs:
        os.environ["SCM_BATCH_PAIRS"] = batch_pairs
    try:
        with Context(0, o_gpu) as ctx:
            ctx.table_load(ids, kps, descs)
            got = ctx.table_run(2, 0, len(imgs))
    finally:
        os.environ.pop("SCM_BATCH_PAIRS", None)
    assert got == ref
    configs = [t.config for row in got[1] for t in decode_tvg_list(row)]
    assert configs.count(8) >= 2
