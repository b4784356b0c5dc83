"""GPU SIFT extraction through the C ABI
(scm_extract_frames) against the CPU oracle (oracle/sift_oracle.cc): the
keypoints, descriptors and camera io.cc elements of
SiftExtractionKernel::execute (extraction_op.cc:70-121) must be the
oracle's byte for byte -- the kernels follow VLFeat's float / double
operation sequence, so the bar is bit-exact, not a tolerance."""
import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd import Context
from scanner_colmap_amd.codecs import decode_descriptors, decode_keypoints
from scanner_colmap_amd.synthetic import synthetic_frame

pytestmark = pytest.mark.gpu


def _diff(got, ref, what):
    if got == ref:
        return ""
    kg, kr = decode_keypoints(got[0]), decode_keypoints(ref[0])
    msg = f"{what}: {len(kg)} vs {len(kr)} keypoints"
    n = min(len(kg), len(kr))
    if n:
        bad = np.nonzero((kg[:n] != kr[:n]).any(axis=1))[0]
        if len(bad):
            msg += f"; first keypoint diff at {bad[0]}: {kg[bad[0]]} vs {kr[bad[0]]}"
        dg, dr = decode_descriptors(got[1])[:n], decode_descriptors(ref[1])[:n]
        bd = np.nonzero((dg != dr).any(axis=1))[0]
        if len(bd):
            msg += (f"; {len(bd)} descriptor rows differ, first {bd[0]}, max |d| "
                    f"{np.abs(dg.astype(int) - dr.astype(int)).max()}")
    if got[2] != ref[2]:
        msg += "; camera differs"
    return msg


@pytest.fixture(scope="module")
def ctx():
    with Context(0) as c:
        yield c


@pytest.mark.parametrize("h,w,ch,seed", [(48, 64, 3, 1), (120, 160, 3, 2), (241, 321, 3, 3),
                                          (97, 130, 1, 4), (200, 150, 4, 5), (480, 640, 3, 6)])
def test_frames_bit_exact(ctx, h, w, ch, seed):
    f = synthetic_frame(h, w, seed, channels=ch)
    got = ctx.extract_frames([f], [1000 + seed])[0]
    ref = oracle.sift_extract(f, 1000 + seed)
    assert got == ref, _diff(got, ref, f"{h}x{w}x{ch}")
    assert len(decode_keypoints(got[0])) > 0


def test_blob_and_batch_of_sizes(ctx):
    """A batch of frames of different sizes (slots reused, workspaces grown)
    in one call, including a single Gaussian blob."""
    yy, xx = np.mgrid[0:96, 0:96].astype(np.float64)
    blob = np.rint(255 * (0.2 + 0.6 * np.exp(-0.5 * ((xx - 48) ** 2 + (yy - 40) ** 2) / 25))).astype(np.uint8)
    frames = [blob, synthetic_frame(300, 400, 11), synthetic_frame(64, 90, 12),
              synthetic_frame(333, 277, 13, channels=1), synthetic_frame(150, 150, 14),
              synthetic_frame(40, 500, 15)]
    got = ctx.extract_frames(frames, list(range(7, 7 + len(frames))))
    for i, f in enumerate(frames):
        ref = oracle.sift_extract(f, 7 + i)
        assert got[i] == ref, _diff(got[i], ref, f"frame {i}")


def test_max_num_features_level_selection(ctx):
    """A frame with more than 8192 keypoints: COLMAP keeps the coarsest DoG
    levels up to and including the one that crosses max_num_features."""
    f = synthetic_frame(1200, 1600, 21, blobs=1600 * 1200 // 150)
    got = ctx.extract_frames([f], [3])[0]
    ref = oracle.sift_extract(f, 3)
    kps = oracle.sift_keypoints(oracle.sift_grey(f))
    assert len(kps) > 8192, len(kps)  # the selection is exercised
    assert got == ref, _diff(got, ref, "1200x1600")
    assert len(decode_keypoints(got[0])) < 2 * len(kps)


def test_extracted_table_feeds_the_matcher(ctx):
    """End to end on the GPU: frames -> extraction rows -> sequential
    matching, equal to the oracle's extraction -> matching."""
    from scanner_colmap_amd.codecs import encode_image_id
    base = synthetic_frame(260, 420, 31)
    frames = [np.ascontiguousarray(base[:, 10 * k: 10 * k + 300]) for k in range(4)]
    rows = ctx.extract_frames(frames, [0, 1, 2, 3])
    ids = [encode_image_id(i) for i in range(4)]
    kps = [r[0] for r in rows]
    descs = [r[1] for r in rows]
    for i, f in enumerate(frames):
        assert rows[i] == oracle.sift_extract(f, i)
    ctx.table_load(ids, kps, descs)
    got_ids, got_tvg = ctx.table_run(3, 0, 4)
    ref_ids, ref_tvg = oracle.table_run(ids, kps, descs, 3, 0, 4)
    assert got_ids == ref_ids and got_tvg == ref_tvg


@pytest.mark.parametrize("h,w,ch,seed", [(2160, 3840, 3, 31),   # 4K: xy order (horizontal first)
                                          (2500, 3300, 3, 32),   # yx order
                                          (60, 3500, 1, 33)])
def test_oversize_frames_rescaled_bit_exact(ctx, h, w, ch, seed):
    # resizeBitmap (extraction_op.cc:28-39): grey, FreeImage bilinear rescale to
    # 3200 / max(w, h), then extraction; camera of the rescaled size
    f = synthetic_frame(h, w, seed, channels=ch, blobs=4000 if h * w > 1e6 else None)
    got = ctx.extract_frames([f, f[:120, :160]], [seed, seed + 1])
    ref = oracle.sift_extract(f, seed)
    assert got[0] == ref, _diff(got[0], ref, f"{h}x{w}x{ch} rescaled")
    assert got[1] == oracle.sift_extract(f[:120, :160], seed + 1)


@pytest.mark.parametrize("h,w,ch", [(15, 40, 3), (40, 15, 1), (9, 9, 4), (5, 7, 3), (1, 1, 1),
                                    (1, 200, 3), (16, 17, 3), (15, 3300, 3)])
def test_tiny_and_thin_frames_bit_exact(ctx, h, w, ch):
    """Frames VLFeat accepts whose octaves have few or no interior pixels
    (the reference has no size floor, extraction_op.cc:71-120), including one
    the max_image_size rescale leaves 14 rows tall: elements byte-equal to
    the oracle's (no keypoints, or a handful, and the camera)."""
    f = np.ascontiguousarray(synthetic_frame(max(h, 64), max(w, 64), 70 + h + w, channels=ch)[:h, :w])
    got = ctx.extract_frames([f], [9])[0]
    ref = oracle.sift_extract(f, 9)
    _diff(got, ref, f"{h}x{w}x{ch}")
    assert got == ref


def test_capacity_overflow_regrows(ctx):
    """Candidate / keypoint / feature capacities far below a frame's needs
    (SCM_SIFT_CAPS): the overflowing frames are extracted again with larger
    capacities, never SCM_E_CAPACITY, and every element equals the oracle's."""
    import os
    from scanner_colmap_amd import Context
    frames = [synthetic_frame(240, 320, 90 + i) for i in range(6)]
    os.environ["SCM_SIFT_CAPS"] = "64,16,16"
    try:
        with Context(0) as c2:
            got = c2.extract_frames(frames, list(range(6)))
    finally:
        del os.environ["SCM_SIFT_CAPS"]
    for i, f in enumerate(frames):
        assert got[i] == oracle.sift_extract(f, i), i
