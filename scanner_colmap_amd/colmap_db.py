"""COLMAP database I/O around the matching stage.

* `read_extraction` turns the `images` / `keypoints` / `descriptors` tables of a
  COLMAP `database.db` into the three columns of the Scanner `extraction`
  table the reference's job reads (`feature_matching.py:61-68`), in the io.cc
  element byte formats (`codecs.py`), so real datasets (Gerrard Hall,
  South-Building) can be matched without Scanner.
* `write_two_view_geometries` stores the op's output rows the way the
  downstream consumer does: `IncrementalMappingCPUKernel::LoadDatabase`
  (reference integration/op_cpp/incremental_mapping.cc:239-262) calls
  `colmap::Database::WriteTwoViewGeometry(pivot, pair_image_ids[k], tvg)` for
  every (pivot row, pair) of `read_two_view_geometries` (io.cc:224-251).

The table layouts follow COLMAP 3.4/3.5's database.cc [upstream, un-vendored]:
image pair id = 2147483647 * min(id1, id2) + max(id1, id2); when the ids are
swapped the geometry is inverted (F and E transposed, H inverted, match
columns swapped); matrices are stored as row-major float64 blobs and matches
as uint32 rows x 2.
"""
from __future__ import annotations

import sqlite3

import numpy as np

from .codecs import (TwoViewGeometry, decode_pair_ids, decode_tvg_list, encode_descriptors,
                     encode_image_id, encode_keypoints)

MAX_NUM_IMAGES = 2147483647  # colmap::kMaxNumImages

SCHEMA = """
CREATE TABLE IF NOT EXISTS cameras (camera_id INTEGER PRIMARY KEY AUTOINCREMENT NOT NULL,
    model INTEGER NOT NULL, width INTEGER NOT NULL, height INTEGER NOT NULL,
    params BLOB, prior_focal_length INTEGER NOT NULL);
CREATE TABLE IF NOT EXISTS images (image_id INTEGER PRIMARY KEY AUTOINCREMENT NOT NULL,
    name TEXT NOT NULL UNIQUE, camera_id INTEGER NOT NULL, prior_qw REAL, prior_qx REAL,
    prior_qy REAL, prior_qz REAL, prior_tx REAL, prior_ty REAL, prior_tz REAL);
CREATE TABLE IF NOT EXISTS keypoints (image_id INTEGER PRIMARY KEY NOT NULL,
    rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB);
CREATE TABLE IF NOT EXISTS descriptors (image_id INTEGER PRIMARY KEY NOT NULL,
    rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB);
CREATE TABLE IF NOT EXISTS matches (pair_id INTEGER PRIMARY KEY NOT NULL,
    rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB);
CREATE TABLE IF NOT EXISTS two_view_geometries (pair_id INTEGER PRIMARY KEY NOT NULL,
    rows INTEGER NOT NULL, cols INTEGER NOT NULL, data BLOB, config INTEGER NOT NULL,
    F BLOB, E BLOB, H BLOB, qvec BLOB, tvec BLOB);
"""


def create_database(path: str) -> sqlite3.Connection:
    """Open (creating if needed) a database with the COLMAP tables used here."""
    con = sqlite3.connect(path)
    con.executescript(SCHEMA)
    return con


def image_pair_to_pair_id(image_id1: int, image_id2: int) -> int:
    """colmap::Database::ImagePairToPairId."""
    if image_id1 > image_id2:
        image_id1, image_id2 = image_id2, image_id1
    return MAX_NUM_IMAGES * image_id1 + image_id2


def pair_id_to_image_pair(pair_id: int) -> tuple[int, int]:
    image_id2 = pair_id % MAX_NUM_IMAGES
    return (pair_id - image_id2) // MAX_NUM_IMAGES, image_id2


def keypoints_to_feature_keypoints(data: np.ndarray) -> np.ndarray:
    """COLMAP keypoint blobs are float32 rows x {2, 4, 6}: (x, y), (x, y, scale,
    orientation) or (x, y, a11, a12, a21, a22) -> FeatureKeypoint rows (x, y,
    a11, a12, a21, a22) as FeatureKeypoint's constructors build them."""
    data = np.asarray(data, np.float32)
    n, cols = data.shape
    out = np.zeros((n, 6), np.float32)
    out[:, :2] = data[:, :2]
    if cols == 2:
        out[:, 2] = 1.0
        out[:, 5] = 1.0
    elif cols == 4:
        scale = data[:, 2].astype(np.float64)
        ori = data[:, 3].astype(np.float64)
        out[:, 2] = scale * np.cos(ori)
        out[:, 3] = -scale * np.sin(ori)
        out[:, 4] = scale * np.sin(ori)
        out[:, 5] = scale * np.cos(ori)
    elif cols == 6:
        out[:, 2:] = data[:, 2:]
    else:
        raise ValueError(f"unsupported keypoint blob with {cols} columns")
    return out


def read_extraction(path: str) -> tuple[list[bytes], list[bytes], list[bytes]]:
    """The `extraction` table columns (image_id, keypoints, descriptors) of every
    image of a COLMAP database, ordered by image_id."""
    con = sqlite3.connect(path)
    try:
        ids, kps, descs = [], [], []
        for (image_id,) in con.execute("SELECT image_id FROM images ORDER BY image_id"):
            row = con.execute("SELECT rows, cols, data FROM keypoints WHERE image_id=?",
                              (image_id,)).fetchone()
            if row is None or not row[0]:
                kp = np.zeros((0, 6), np.float32)
            else:
                kp = keypoints_to_feature_keypoints(
                    np.frombuffer(row[2], np.float32).reshape(row[0], row[1]))
            row = con.execute("SELECT rows, cols, data FROM descriptors WHERE image_id=?",
                              (image_id,)).fetchone()
            if row is None or not row[0]:
                d = np.zeros((0, 128), np.uint8)
            else:
                if row[1] != 128:
                    raise ValueError(f"image {image_id}: {row[1]}-D descriptors, expected 128")
                d = np.frombuffer(row[2], np.uint8).reshape(row[0], 128)
            if len(d) != len(kp):
                raise ValueError(f"image {image_id}: {len(kp)} keypoints, {len(d)} descriptors")
            ids.append(encode_image_id(int(image_id)))
            kps.append(encode_keypoints(kp))
            descs.append(encode_descriptors(d))
        return ids, kps, descs
    finally:
        con.close()


def _inverted(tvg: TwoViewGeometry) -> TwoViewGeometry:
    """colmap::TwoViewGeometry::Invert for a swapped image pair."""
    H = np.asarray(tvg.H, np.float64)
    try:
        Hinv = np.linalg.inv(H) if np.any(H) else H
    except np.linalg.LinAlgError:
        Hinv = H
    m = np.asarray(tvg.inlier_matches, np.uint32).reshape(-1, 2)
    return TwoViewGeometry(config=tvg.config, E=np.asarray(tvg.E).T.copy(),
                           F=np.asarray(tvg.F).T.copy(), H=Hinv, qvec=tvg.qvec, tvec=tvg.tvec,
                           tri_angle=tvg.tri_angle, inlier_matches=m[:, ::-1].copy())


def write_two_view_geometry(con: sqlite3.Connection, image_id1: int, image_id2: int,
                            tvg: TwoViewGeometry) -> None:
    """colmap::Database::WriteTwoViewGeometry."""
    if image_id1 > image_id2:
        tvg = _inverted(tvg)
    m = np.ascontiguousarray(np.asarray(tvg.inlier_matches, np.uint32).reshape(-1, 2))
    mat = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).reshape(3, 3)).tobytes()
    con.execute("INSERT OR REPLACE INTO two_view_geometries VALUES (?,?,?,?,?,?,?,?,?,?)",
                (image_pair_to_pair_id(image_id1, image_id2), len(m), 2,
                 m.tobytes() if len(m) else None, int(tvg.config), mat(tvg.F), mat(tvg.E),
                 mat(tvg.H), np.asarray(tvg.qvec, np.float64).tobytes(),
                 np.asarray(tvg.tvec, np.float64).tobytes()))


def write_two_view_geometries(path: str, pivot_ids: list[int], pair_rows: list[bytes],
                              tvg_rows: list[bytes]) -> int:
    """Store the op's output rows (pair_image_ids + two_view_geometries
    elements per pivot row) as LoadDatabase does; returns the pair count."""
    con = create_database(path)
    try:
        count = 0
        for pivot, pa, pb in zip(pivot_ids, pair_rows, tvg_rows):
            ids = decode_pair_ids(pa)
            tvgs = decode_tvg_list(pb)
            if len(ids) != len(tvgs):  # CHECK_EQ in LoadDatabase
                raise ValueError(f"pivot {pivot}: {len(ids)} pair ids, {len(tvgs)} geometries")
            for j, tvg in zip(ids, tvgs):
                write_two_view_geometry(con, int(pivot), int(j), tvg)
                count += 1
        con.commit()
        return count
    finally:
        con.close()


def read_two_view_geometry(path: str, image_id1: int, image_id2: int) -> TwoViewGeometry | None:
    """Read one geometry back in (image_id1, image_id2) orientation."""
    con = sqlite3.connect(path)
    try:
        row = con.execute("SELECT rows, cols, data, config, F, E, H, qvec, tvec FROM "
                          "two_view_geometries WHERE pair_id=?",
                          (image_pair_to_pair_id(image_id1, image_id2),)).fetchone()
    finally:
        con.close()
    if row is None:
        return None
    rows, cols, data, config, F, E, H, qvec, tvec = row
    m = (np.frombuffer(data, np.uint32).reshape(rows, cols) if rows
         else np.zeros((0, 2), np.uint32))
    mat = lambda b: np.frombuffer(b, np.float64).reshape(3, 3).copy()
    tvg = TwoViewGeometry(config=int(config), F=mat(F), E=mat(E), H=mat(H),
                          qvec=np.frombuffer(qvec, np.float64).copy(),
                          tvec=np.frombuffer(tvec, np.float64).copy(), inlier_matches=m)
    return _inverted(tvg) if image_id1 > image_id2 else tvg


def write_extraction_database(path: str, images) -> None:
    """Test / tooling helper: a COLMAP database holding synthetic images
    ((image_id, FeatureKeypoint rows, descriptors) tuples, e.g. from
    synthetic.Corridor), with 6-column keypoint blobs."""
    con = create_database(path)
    try:
        con.execute("INSERT OR IGNORE INTO cameras VALUES (1, 0, 1920, 1080, ?, 0)",
                    (np.array([1000.0, 960.0, 540.0], np.float64).tobytes(),))
        for image_id, kp, d in images:
            kp = np.asarray(kp, np.float32).reshape(-1, 6)
            d = np.asarray(d, np.uint8).reshape(-1, 128)
            con.execute("INSERT INTO images (image_id, name, camera_id) VALUES (?,?,1)",
                        (int(image_id), f"img{int(image_id):06d}.jpg"))
            con.execute("INSERT INTO keypoints VALUES (?,?,?,?)",
                        (int(image_id), len(kp), 6, kp.tobytes()))
            con.execute("INSERT INTO descriptors VALUES (?,?,?,?)",
                        (int(image_id), len(d), 128, d.tobytes()))
        con.commit()
    finally:
        con.close()


__all__ = ["create_database", "image_pair_to_pair_id", "pair_id_to_image_pair",
           "keypoints_to_feature_keypoints", "read_extraction", "write_two_view_geometry",
           "write_two_view_geometries", "read_two_view_geometry", "write_extraction_database",
           "MAX_NUM_IMAGES"]
