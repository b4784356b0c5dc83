"""Known answers for the SIFT extraction oracle (oracle/sift_oracle.cc, SURVEY.md
§8f rank 4: SiftExtractionKernel::execute, extraction_op.cc:70-121, which
drives colmap::ExtractSiftFeaturesCPU -> VLFeat vl/sift.c).  FreeImage,
VLFeat and COLMAP are absent and the reference ships no fixtures, so the
oracle is parity unpinned; these tests pin it to the published algorithm:
the vl/mathop.h approximations against their exact functions, the Gaussian
scale space against an independent numpy restatement, a single blob's
keypoint position and scale, the L1-root descriptor norm, 90-degree rotation
covariance, and the io.cc element layouts."""
import struct

import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd.codecs import decode_descriptors, decode_keypoints
from scanner_colmap_amd.synthetic import synthetic_frame


def test_mathop_approximations():
    atan2, fsqrt, expn, taps = oracle.sift_math()
    rng = np.random.default_rng(0)
    for _ in range(2000):
        y, x = rng.normal(size=2) * rng.uniform(0.01, 10)
        a = atan2(float(y), float(x))
        assert abs(a - np.arctan2(y, x)) < 0.0065  # vl_fast_atan2_f: cubic in r, |err| <~ 0.0062 rad
        v = float(rng.uniform(1e-6, 100))
        assert abs(fsqrt(v) - np.sqrt(v)) <= 1e-5 * np.sqrt(v)
    assert fsqrt(1e-9) == 0.0  # vl_fast_sqrt_f returns 0 below 1e-8
    for x in np.linspace(0, 24.9, 500):
        assert abs(expn(float(x)) - np.exp(-x)) < 2.5e-3  # linear interpolation of 257 samples
    assert expn(25.5) == 0.0
    for sigma in (1.2489995996796797, 1.2262735, 1.5450, 1.9466, 2.4525, 3.0900):
        g = taps(sigma)
        W = max(int(np.ceil(4 * sigma)), 1)
        assert len(g) == 2 * W + 1
        assert (g == g[::-1]).all()
        assert abs(float(g.astype(np.float64).sum()) - 1.0) < 1e-6
        ref = np.exp(-0.5 * ((np.arange(-W, W + 1) / sigma) ** 2))
        assert np.allclose(g, ref / ref.sum(), rtol=1e-6, atol=1e-9)


def _np_smooth(img, sigma):
    W = max(int(np.ceil(4 * sigma)), 1)
    g = np.exp(-0.5 * ((np.arange(-W, W + 1) / sigma) ** 2))
    g /= g.sum()
    p = np.pad(img, ((W, W), (0, 0)), mode="edge")
    v = sum(g[W + k] * p[W + k: W + k + img.shape[0], :] for k in range(-W, W + 1))
    p = np.pad(v, ((0, 0), (W, W)), mode="edge")
    return sum(g[W + k] * p[:, W + k: W + k + img.shape[1]] for k in range(-W, W + 1))


def test_scale_space_matches_numpy_restatement():
    grey = oracle.sift_grey(synthetic_frame(60, 80, 3))
    oc = oracle.sift_octave(grey, -1)
    assert oc.shape == (6, 120, 160)
    im = grey.astype(np.float64) / 255.0
    h, w = im.shape
    # copy_and_upsample_rows twice: x, then y (last sample repeated)
    up = np.zeros((h, 2 * w))
    up[:, 0::2] = im
    up[:, 1::2] = np.concatenate([(im[:, :-1] + im[:, 1:]) / 2, im[:, -1:]], axis=1)
    up2 = np.zeros((2 * h, 2 * w))
    up2[0::2] = up
    up2[1::2] = np.concatenate([(up[:-1] + up[1:]) / 2, up[-1:]], axis=0)
    k = 2 ** (1 / 3)
    s0 = 1.6 * k
    lev = _np_smooth(up2, np.sqrt((s0 / k) ** 2 - 1.0))
    ref = [lev]
    for s in range(0, 5):
        lev = _np_smooth(lev, s0 * np.sqrt(1 - 1 / k ** 2) * k ** s)
        ref.append(lev)
    assert np.abs(oc - np.stack(ref)).max() < 2e-6
    # next octave: level s = 2 subsampled, no extra smoothing (sa == sb)
    o0 = oracle.sift_octave(grey, 0)
    assert o0.shape == (6, 60, 80)
    assert (o0[0] == oc[3][0::2, 0::2]).all()


def _blob(h, w, cx, cy, sigma, amp=0.6):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = 0.2 + amp * np.exp(-0.5 * ((xx - cx) ** 2 + (yy - cy) ** 2) / sigma ** 2)
    return np.rint(np.clip(img, 0, 1) * 255).astype(np.uint8)


@pytest.mark.parametrize("sigma", [3.0, 5.0, 8.0])
def test_single_blob_keypoint(sigma):
    """An isotropic Gaussian blob of std sigma: a keypoint at its centre
    (pixel (i, j) -> COLMAP (i + 0.5, j + 0.5)) at scale ~ 0.9 sigma (the
    scale-normalised Laplacian of a Gaussian blob peaks at sigma; the sampled
    levels sit a little below).  The centre lies on the pixel grid of every
    octave: a centre between grid points makes a 2 x 2 plateau of equal DoG
    values, which VLFeat's strict 26-neighbour test rejects."""
    g = _blob(96, 96, 48.0, 40.0, sigma)
    kps = oracle.sift_keypoints(g)
    assert len(kps) >= 1
    d = np.hypot(kps[:, 4] - 48.0, kps[:, 5] - 40.0)
    best = kps[np.argmin(d)]
    assert d.min() < 0.05
    assert abs(best[6] / sigma - 0.9) < 0.15
    f = np.repeat(g[:, :, None], 3, axis=2)
    kb, db, _ = oracle.sift_extract(f)
    kp = decode_keypoints(kb)
    assert np.hypot(kp[:, 0] - 48.5, kp[:, 1] - 40.5).min() < 0.05


def test_descriptor_and_keypoint_layout():
    f = synthetic_frame(200, 260, 5)
    kb, db, cb = oracle.sift_extract(f, image_id=12345)
    kp = decode_keypoints(kb)
    d = decode_descriptors(db).astype(np.float64)
    assert len(kp) == len(d) > 50
    assert (kp[:, 0] >= 0.5).all() and (kp[:, 0] <= 259.5).all()
    # L1-root descriptors have unit L2 norm before the x512 quantisation
    n2 = (d ** 2).sum(axis=1)
    assert np.abs(np.sqrt(n2) / 512 - 1).max() < 0.05
    # affine part = scale * rotation (FeatureKeypoint(x, y, scale, orientation))
    sc = np.hypot(kp[:, 2], kp[:, 4])
    assert np.allclose(kp[:, 3], -kp[:, 4], atol=1e-5) and np.allclose(kp[:, 5], kp[:, 2], atol=1e-5)
    assert (sc >= 0.5 * 1.6 - 1e-6).all()  # smallest VLFeat scale: sigma0 2^(s_min / 3) xper = 1.6 x 0.5
    # camera element (io.cc:307-333): SIMPLE_RADIAL f = 1.2 max(w, h), (w/2, h/2), k = 0
    tot, cid, model, w, h, prior, npar = struct.unpack_from("<QIiQQ?Q", cb, 0)
    params = struct.unpack_from("<4d", cb, 8 + 4 + 4 + 8 + 8 + 1 + 8)
    assert tot == len(cb) == 73 and cid == 12345 and model == 2 and (w, h) == (260, 200)
    assert not prior and npar == 4 and params == (312.0, 130.0, 100.0, 0.0)


def test_grey_conversion_bgr_memory_order():
    """FreeImage_ConvertFromRawBits keeps the frame bytes as FreeImage's B, G,
    R memory order, so frame channel 2 carries the red weight 0.2126."""
    rng = np.random.default_rng(3)
    f = rng.integers(0, 256, (7, 9, 3), dtype=np.uint8)
    g = oracle.sift_grey(f)
    ff = f.astype(np.float32)
    ref = (np.float32(0.2126) * ff[:, :, 2] + np.float32(0.7152) * ff[:, :, 1]
           + np.float32(0.0722) * ff[:, :, 0] + np.float32(0.5)).astype(np.uint8)
    assert (g == ref).all()
    f4 = np.concatenate([f, np.full((7, 9, 1), 9, np.uint8)], axis=2)
    assert (oracle.sift_grey(f4) == g).all()
    assert (oracle.sift_grey(f[:, :, :1]) == f[:, :, 0]).all()


def test_rotation_covariance():
    """A 90-degree rotation of the frame rotates keypoints and orientations
    and (the descriptor being relative to the orientation) keeps most
    descriptors close."""
    f = synthetic_frame(160, 160, 9)
    k0 = decode_keypoints(oracle.sift_extract(f)[0])
    d0 = decode_descriptors(oracle.sift_extract(f)[1]).astype(np.float64)
    r = np.ascontiguousarray(np.rot90(f, k=-1))  # clockwise: (x, y) -> (H - 1 - y, x) in pixel centres
    k1 = decode_keypoints(oracle.sift_extract(r)[0])
    d1 = decode_descriptors(oracle.sift_extract(r)[1]).astype(np.float64)
    # pixel corners convention (+0.5): x' = H - y, y' = x
    px = np.stack([160 - k0[:, 1], k0[:, 0]], axis=1)
    hits = 0
    for i in range(len(k0)):
        dd = np.hypot(k1[:, 0] - px[i, 0], k1[:, 1] - px[i, 1])
        j = np.argmin(dd)
        if dd[j] < 0.5 and np.linalg.norm(d0[i] - d1[j]) < 0.25 * 512:
            hits += 1
    assert hits > 0.6 * len(k0), (hits, len(k0))


@pytest.mark.parametrize("w,h", [(3840, 2160), (3300, 2500), (3200, 3200), (20, 3201),
                                 (5000, 3333), (100, 100), (3201, 3201)])
def test_fit_size_is_resize_bitmap(w, h):
    # extraction_op.cc:28-39: scale = 3200 / max(w, h), sizes truncated (C double arithmetic)
    if w > 3200 or h > 3200:
        s = 3200.0 / max(w, h)
        want = (int(w * s), int(h * s))
    else:
        want = (w, h)
    assert oracle.sift_fit_size(w, h) == want


def test_rescale_known_answers():
    rng = np.random.default_rng(11)
    # constant image, and identity size
    assert (oracle.sift_rescale(np.full((30, 50), 77, np.uint8), 37, 21) == 77).all()
    g = rng.integers(0, 256, (33, 47), dtype=np.uint8)
    assert (oracle.sift_rescale(g, 47, 33) == g).all()
    # exact 2:1 minification: bilinear (width 1) stretched by 2 gives the taps
    # 1/8, 3/8, 3/8, 1/8 on source pixels 2u-1 .. 2u+2 (exact in fp64)
    row = rng.integers(0, 256, 64).astype(np.float64)
    r = oracle.sift_rescale(np.repeat(row[None, :].astype(np.uint8), 6, 0), 32, 3)
    want = [int(0.125 * row[2 * u - 1] + 0.375 * row[2 * u] + 0.375 * row[2 * u + 1]
                + 0.125 * row[2 * u + 2] + 0.5) for u in range(1, 31)]
    assert (r[:, 1:31] == np.array(want)).all()
    col = rng.integers(0, 256, 64).astype(np.float64)
    r = oracle.sift_rescale(np.repeat(col[:, None].astype(np.uint8), 6, 1), 3, 32)
    want = [int(0.125 * col[2 * u - 1] + 0.375 * col[2 * u] + 0.375 * col[2 * u + 1]
                + 0.125 * col[2 * u + 2] + 0.5) for u in range(1, 31)]
    assert (r[1:31, :] == np.array(want)[:, None]).all()
    # first pixel: the window is clipped at the border and renormalised by its
    # total 7/8 (FreeImage divides each weight, then sums in source order)
    v = 0.0
    for wgt, c in zip((0.375 / 0.875, 0.375 / 0.875, 0.125 / 0.875), col[:3]):
        v += wgt * c
    assert r[0, 0] == int(v + 0.5)


def test_oversize_frame_is_rescaled_before_extraction():
    # resizeBitmap then extraction == extraction of the rescaled grey image
    f = synthetic_frame(40, 3300, 21)
    nw, nh = oracle.sift_fit_size(3300, 40)
    small = oracle.sift_rescale(oracle.sift_grey(f), nw, nh)
    got = oracle.sift_extract(f, 5)
    assert got == oracle.sift_extract(small[:, :, None], 5)
    assert np.frombuffer(got[2][16:32], np.uint64).tolist() == [nw, nh]  # camera: rescaled size
    # 14 rows after the rescale: VLFeat runs on it like on any size (no floor)
    thin = oracle.sift_extract(np.zeros((15, 3300, 3), np.uint8))
    assert np.frombuffer(thin[2][16:32], np.uint64).tolist() == [3200, 14]


def test_refine_terms_round_sums_in_float():
    """vl_sift_refine_keypoints' at() reads vl_sift_pix (float), so in
    `Dx = 0.5 * (at(+1,0,0) - at(-1,0,0))` the difference rounds in float and
    only the product with the double literal widens (C's usual arithmetic
    conversions; same for the Hessian sums).  Known answer from numpy float32
    arithmetic on patches where evaluating the sums in double would differ."""
    import ctypes
    from oracle import oracle
    L = oracle.lib()
    L.oracle_sift_refine_terms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(5)
    f = np.float32
    differs = 0
    for _ in range(200):
        p = (rng.uniform(-0.05, 0.05, (3, 3, 3)) * rng.uniform(0.5, 3.0)).astype(np.float32)
        out = np.zeros(9, np.float64)
        L.oracle_sift_refine_terms(p.ctypes.data, out.ctypes.data)

        def a(dx, dy, ds):
            return p[1 + ds, 1 + dy, 1 + dx]
        ref = [0.5 * np.float64(f(a(1, 0, 0) - a(-1, 0, 0))),
               0.5 * np.float64(f(a(0, 1, 0) - a(0, -1, 0))),
               0.5 * np.float64(f(a(0, 0, 1) - a(0, 0, -1))),
               np.float64(f(a(1, 0, 0) + a(-1, 0, 0))) - 2.0 * np.float64(a(0, 0, 0)),
               np.float64(f(a(0, 1, 0) + a(0, -1, 0))) - 2.0 * np.float64(a(0, 0, 0)),
               np.float64(f(a(0, 0, 1) + a(0, 0, -1))) - 2.0 * np.float64(a(0, 0, 0)),
               0.25 * np.float64(f(f(f(a(1, 1, 0) + a(-1, -1, 0)) - a(-1, 1, 0)) - a(1, -1, 0))),
               0.25 * np.float64(f(f(f(a(1, 0, 1) + a(-1, 0, -1)) - a(-1, 0, 1)) - a(1, 0, -1))),
               0.25 * np.float64(f(f(f(a(0, 1, 1) + a(0, -1, -1)) - a(0, -1, 1)) - a(0, 1, -1)))]
        assert out.tolist() == ref
        d = np.float64
        dbl = [0.5 * (d(a(1, 0, 0)) - d(a(-1, 0, 0))),
               0.25 * (d(a(1, 1, 0)) + d(a(-1, -1, 0)) - d(a(-1, 1, 0)) - d(a(1, -1, 0)))]
        differs += (dbl[0] != ref[0]) + (dbl[1] != ref[6])
    assert differs > 50  # the patches do tell float from double sums apart
