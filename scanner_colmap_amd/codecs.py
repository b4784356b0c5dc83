"""Python encoders / decoders of the reference's Scanner element byte formats
(reference integration/op_cpp/io.cc).

Used by the job-script mirror (feature_matching.py), the tests and the
benchmark to build `extraction`-table rows and to read `matching`-table rows.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("a11", "<f4"),
                           ("a12", "<f4"), ("a21", "<f4"), ("a22", "<f4")])


def encode_image_id(image_id: int) -> bytes:
    """prepare_image.cc:17-20 writes the id as size_t (read back as the low
    4 bytes by read_single_from_element<image_t>, io.cc:67-69)."""
    return struct.pack("<Q", image_id)


def encode_keypoints(kp: np.ndarray) -> bytes:
    """write_vector_to_element<FeatureKeypoints> (io.cc:151-169):
    size_t n + n x FeatureKeypoint{float x, y, a11, a12, a21, a22}."""
    kp = np.ascontiguousarray(kp, dtype=np.float32).reshape(-1, 6)
    return struct.pack("<Q", len(kp)) + kp.tobytes()


def decode_keypoints(b: bytes) -> np.ndarray:
    (n,) = struct.unpack_from("<Q", b, 0)
    return np.frombuffer(b, dtype=np.float32, count=6 * n, offset=8).reshape(n, 6)


def encode_descriptors(d: np.ndarray) -> bytes:
    """write_matrix_to_element<FeatureDescriptors> (io.cc:196-219):
    size_t rows, size_t cols, row-major uint8."""
    d = np.ascontiguousarray(d, dtype=np.uint8).reshape(-1, 128)
    return struct.pack("<QQ", d.shape[0], d.shape[1]) + d.tobytes()


def decode_descriptors(b: bytes) -> np.ndarray:
    rows, cols = struct.unpack_from("<QQ", b, 0)
    return np.frombuffer(b, dtype=np.uint8, count=rows * cols, offset=16).reshape(rows, cols)


def decode_pair_ids(b: bytes) -> list[int]:
    """createVectorBuffer<vector<image_t>> (io.cc:151-162)."""
    (n,) = struct.unpack_from("<Q", b, 0)
    return list(np.frombuffer(b, dtype=np.uint32, count=n, offset=8))


TVG_HEADER = struct.Struct("<i9d9d9d4d3dd")   # config, E, F, H, qvec, tvec, tri_angle
assert TVG_HEADER.size == 4 + 8 * 35


@dataclass
class TwoViewGeometry:
    config: int = 0
    E: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))
    F: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))
    H: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))
    qvec: np.ndarray = field(default_factory=lambda: np.zeros(4))
    tvec: np.ndarray = field(default_factory=lambda: np.zeros(3))
    tri_angle: float = 0.0
    inlier_matches: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.uint32))


def _decode_one_tvg(b: bytes, off: int) -> tuple[TwoViewGeometry, int]:
    v = TVG_HEADER.unpack_from(b, off)
    off += TVG_HEADER.size
    t = TwoViewGeometry()
    t.config = v[0]
    # Eigen::Matrix3d is column-major in memory.
    t.E = np.array(v[1:10]).reshape(3, 3).T
    t.F = np.array(v[10:19]).reshape(3, 3).T
    t.H = np.array(v[19:28]).reshape(3, 3).T
    t.qvec = np.array(v[28:32])
    t.tvec = np.array(v[32:35])
    t.tri_angle = v[35]
    (n,) = struct.unpack_from("<Q", b, off)
    off += 8
    t.inlier_matches = np.frombuffer(b, dtype=np.uint32, count=2 * n, offset=off).reshape(n, 2)
    off += 8 * n
    return t, off


def decode_tvg(b: bytes) -> TwoViewGeometry:
    """One TVG in the per-geometry layout of io.cc:279-292."""
    t, off = _decode_one_tvg(b, 0)
    assert off == len(b), (off, len(b))
    return t


def decode_tvg_list(b: bytes) -> list[TwoViewGeometry]:
    """read_two_view_geometries (io.cc:224-251): size_t total, int count."""
    total, count = struct.unpack_from("<Qi", b, 0)
    assert total == len(b), (total, len(b))
    off = 12
    out = []
    for _ in range(count):
        t, off = _decode_one_tvg(b, off)
        out.append(t)
    assert off == total
    return out


def split_tvg_list(b: bytes) -> list[bytes]:
    """The per-TVG byte ranges of a two_view_geometries element (io.cc:256-297):
    each TVG is 292 B + 8 B per inlier match."""
    total, count = struct.unpack_from("<Qi", b, 0)
    assert total == len(b), (total, len(b))
    off = 12
    out = []
    for _ in range(count):
        (n,) = struct.unpack_from("<Q", b, off + TVG_HEADER.size)
        end = off + TVG_HEADER.size + 8 + 8 * n
        out.append(bytes(b[off:end]))
        off = end
    assert off == total
    return out


def encode_tvg_list(tvgs: list[TwoViewGeometry]) -> bytes:
    """create_two_view_geometries_buffer (io.cc:256-297)."""
    body = b""
    for t in tvgs:
        m = np.ascontiguousarray(t.inlier_matches, dtype=np.uint32).reshape(-1, 2)
        body += TVG_HEADER.pack(int(t.config), *np.asarray(t.E).T.reshape(-1),
                                *np.asarray(t.F).T.reshape(-1), *np.asarray(t.H).T.reshape(-1),
                                *np.asarray(t.qvec).reshape(-1), *np.asarray(t.tvec).reshape(-1),
                                float(t.tri_angle))
        body += struct.pack("<Q", len(m)) + m.tobytes()
    return struct.pack("<Qi", 12 + len(body), len(tvgs)) + body


def table_rows(images) -> tuple[list[bytes], list[bytes], list[bytes]]:
    """Encode a list of (image_id, keypoints N x 6, descriptors N x 128) as the
    three `extraction`-table columns the matcher reads
    (feature_matching.py:61-68)."""
    ids, kps, descs = [], [], []
    for image_id, kp, d in images:
        ids.append(encode_image_id(image_id))
        kps.append(encode_keypoints(kp))
        descs.append(encode_descriptors(d))
    return ids, kps, descs
