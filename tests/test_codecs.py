"""io.cc byte formats and the sequential pair
schedule (a17), checked on the CPU oracle's output rows."""
import struct

import numpy as np

from oracle import oracle
from scanner_colmap_amd.codecs import (TVG_HEADER, TwoViewGeometry, decode_descriptors,
                                       decode_keypoints, decode_pair_ids, decode_tvg_list,
                                       encode_descriptors, encode_image_id, encode_keypoints,
                                       encode_tvg_list, table_rows)
from scanner_colmap_amd.distributed import pairs_per_row
from scanner_colmap_amd.synthetic import Corridor


def test_element_layouts():
    kp = np.arange(12, dtype=np.float32).reshape(2, 6)
    b = encode_keypoints(kp)
    assert len(b) == 8 + 48 and struct.unpack_from("<Q", b)[0] == 2
    assert (decode_keypoints(b) == kp).all()
    d = np.arange(256, dtype=np.uint8).reshape(2, 128)
    b = encode_descriptors(d)
    assert struct.unpack_from("<QQ", b) == (2, 128) and len(b) == 16 + 256
    assert (decode_descriptors(b) == d).all()
    assert encode_image_id(7) == (7).to_bytes(8, "little")


def test_tvg_layout_known_bytes():
    t = TwoViewGeometry(config=3)
    t.F = np.arange(9, dtype=float).reshape(3, 3)
    t.H = -np.arange(9, dtype=float).reshape(3, 3)
    t.inlier_matches = np.array([[1, 2], [3, 4]], np.uint32)
    b = encode_tvg_list([t])
    assert len(b) == 12 + 292 + 16
    total, count = struct.unpack_from("<Qi", b)
    assert (total, count) == (len(b), 1)
    assert struct.unpack_from("<i", b, 12)[0] == 3
    # F column-major at config + E: F(1,0) = 3 is the second double
    f = struct.unpack_from("<9d", b, 12 + 4 + 72)
    assert f == (0.0, 3.0, 6.0, 1.0, 4.0, 7.0, 2.0, 5.0, 8.0)
    assert struct.unpack_from("<Q", b, 12 + TVG_HEADER.size)[0] == 2
    assert struct.unpack_from("<4I", b, 12 + TVG_HEADER.size + 8) == (1, 2, 3, 4)
    back = decode_tvg_list(b)[0]
    assert back.config == 3 and (back.F == t.F).all() and (back.H == t.H).all()
    assert encode_tvg_list([]) == struct.pack("<Qi", 12, 0)


def test_oracle_rows_round_trip_and_schedule():
    n, K = 7, 4
    imgs = Corridor(n, 500, K, seed=29).images()
    ids, kps, descs = table_rows(imgs)
    pa, pb = oracle.table_run(ids, kps, descs, K, 0, n)
    ppr = pairs_per_row(n, K)
    for r in range(n):
        want = [imgs[j][0] for j in range(r + 1, min(r + K, n))]
        assert decode_pair_ids(pa[r]) == want
        assert len(want) == ppr[r]
        tv = decode_tvg_list(pb[r])
        assert len(tv) == len(want)
        assert encode_tvg_list(tv) == pb[r]
        for t in tv:
            if t.config == 0:
                assert len(t.inlier_matches) == 0
            else:
                assert len(t.inlier_matches) >= 15
    assert pb[-1] == struct.pack("<Qi", 12, 0)  # the empty last row is 12 B
    assert pa[-1] == struct.pack("<Q", 0)


def test_stencil_dedups_repeated_ids():
    """sequential_matching.cc:141-144: stencil entries equal to the pivot id
    or already paired are skipped (this is what neutralises clamping)."""
    imgs = Corridor(4, 300, 4, seed=31).images()
    ids, kps, descs = table_rows(imgs)
    sel = [0, 1, 1, 0, 2]
    a, b = oracle.execute_stencil([ids[i] for i in sel], [kps[i] for i in sel],
                                  [descs[i] for i in sel])
    assert decode_pair_ids(a) == [imgs[1][0], imgs[2][0]]
    assert len(decode_tvg_list(b)) == 2
