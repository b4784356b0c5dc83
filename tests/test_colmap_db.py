"""COLMAP database I/O around the stage (scanner_colmap_amd/colmap_db.py,
SURVEY.md §8f ranks 2-3): extraction rows read from a database.db and the
op's output rows stored the way IncrementalMappingCPUKernel::LoadDatabase
stores them (reference incremental_mapping.cc:239-262)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from scanner_colmap_amd import colmap_db
from scanner_colmap_amd.codecs import decode_pair_ids, decode_tvg_list, table_rows
from scanner_colmap_amd.synthetic import Corridor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pair_id_roundtrip():
    for a, b in ((1, 2), (2, 1), (7, 7), (2147483646, 3)):
        pid = colmap_db.image_pair_to_pair_id(a, b)
        assert colmap_db.pair_id_to_image_pair(pid) == (min(a, b), max(a, b))
    assert colmap_db.image_pair_to_pair_id(1, 2) == 2147483647 + 2


def test_keypoint_blob_layouts():
    xy = np.array([[1.5, 2.5], [3.0, 4.0]], np.float32)
    k2 = colmap_db.keypoints_to_feature_keypoints(xy)
    assert np.array_equal(k2, [[1.5, 2.5, 1, 0, 0, 1], [3, 4, 1, 0, 0, 1]])
    k4 = colmap_db.keypoints_to_feature_keypoints(np.array([[1, 2, 2.0, np.pi / 2]], np.float32))
    assert np.allclose(k4, [[1, 2, 0, -2, 2, 0]], atol=1e-6)
    k6 = np.arange(12, dtype=np.float32).reshape(2, 6)
    assert np.array_equal(colmap_db.keypoints_to_feature_keypoints(k6), k6)
    with pytest.raises(ValueError):
        colmap_db.keypoints_to_feature_keypoints(np.zeros((1, 3), np.float32))


def test_read_extraction_equals_table_rows(tmp_path):
    imgs = Corridor(4, 300, 3, seed=61).images()
    db = str(tmp_path / "db.db")
    colmap_db.write_extraction_database(db, imgs)
    assert colmap_db.read_extraction(db) == tuple(table_rows(imgs))


def test_write_two_view_geometries_as_load_database(tmp_path):
    from oracle import oracle
    imgs = Corridor(5, 500, 4, seed=62).images()
    ids, kps, descs = table_rows(imgs)
    pa, pb = oracle.table_run(ids, kps, descs, 4, 0, len(ids))
    db = str(tmp_path / "out.db")
    pivots = [im[0] for im in imgs]
    n = colmap_db.write_two_view_geometries(db, pivots, pa, pb)
    assert n == sum(len(decode_pair_ids(x)) for x in pa)
    for pivot, a, b in zip(pivots, pa, pb):
        for j, tvg in zip(decode_pair_ids(a), decode_tvg_list(b)):
            got = colmap_db.read_two_view_geometry(db, pivot, int(j))
            assert got.config == tvg.config
            assert np.array_equal(got.F, tvg.F) and np.array_equal(got.H, tvg.H)
            assert np.array_equal(got.inlier_matches, np.asarray(tvg.inlier_matches).reshape(-1, 2))


def test_swapped_pair_is_stored_inverted(tmp_path):
    from scanner_colmap_amd.codecs import TwoViewGeometry
    rng = np.random.default_rng(3)
    tvg = TwoViewGeometry(config=3, F=rng.normal(size=(3, 3)), H=rng.normal(size=(3, 3)),
                          inlier_matches=np.array([[1, 5], [2, 7]], np.uint32))
    db = str(tmp_path / "s.db")
    con = colmap_db.create_database(db)
    colmap_db.write_two_view_geometry(con, 9, 4, tvg)  # pivot id above the neighbour's
    con.commit()
    con.close()
    stored = colmap_db.read_two_view_geometry(db, 4, 9)
    assert np.array_equal(stored.F, tvg.F.T)
    assert np.allclose(stored.H, np.linalg.inv(tvg.H))
    assert np.array_equal(stored.inlier_matches, [[5, 1], [7, 2]])
    back = colmap_db.read_two_view_geometry(db, 9, 4)
    assert np.array_equal(back.F, tvg.F) and np.allclose(back.H, tvg.H)
    assert np.array_equal(back.inlier_matches, tvg.inlier_matches)


@pytest.mark.gpu
def test_feature_matching_cli_end_to_end(tmp_path):
    """The job-script mirror on a COLMAP database: GPU rows written to the
    output database equal the oracle's rows for the same extraction table."""
    from oracle import oracle
    imgs = Corridor(6, 700, 4, seed=63).images()
    src = str(tmp_path / "in.db")
    out = str(tmp_path / "out.db")
    colmap_db.write_extraction_database(src, imgs)
    r = subprocess.run([sys.executable, "-m", "scanner_colmap_amd.feature_matching", "--database",
                        src, "--output_database", out, "--overlap", "4"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ids, kps, descs = colmap_db.read_extraction(src)
    pa, pb = oracle.table_run(ids, kps, descs, 4, 0, len(ids))
    for im, a, b in zip(imgs, pa, pb):
        for j, tvg in zip(decode_pair_ids(a), decode_tvg_list(b)):
            got = colmap_db.read_two_view_geometry(out, im[0], int(j))
            assert got.config == tvg.config
            assert np.array_equal(got.F, tvg.F) and np.array_equal(got.H, tvg.H)
            assert np.array_equal(got.inlier_matches, np.asarray(tvg.inlier_matches).reshape(-1, 2))
