"""Deterministic synthetic `extraction` tables (SURVEY.md §8d "Synthetic
inputs"): a camera moving along a corridor of 3-D points, each image seeing a
sliding window of the points so that its overlap with the next image decays
over about `overlap` images; keypoints are noisy projections plus uniform
outliers; descriptors are per-point base vectors perturbed per view and
RootSIFT-normalised to uint8 like COLMAP's extractor output
(min(255, round(512 * v))).

No dataset or checkpoint is downloaded anywhere; every configuration of
BASELINE.json is generated from a seed.
"""
from __future__ import annotations

import numpy as np


def rootsift_u8(v: np.ndarray) -> np.ndarray:
    """L1-normalise, sqrt, L2-normalise, u8 = min(255, round(512 v))."""
    v = np.abs(v).astype(np.float32)
    v /= np.maximum(v.sum(axis=1, keepdims=True), 1e-12)
    v = np.sqrt(v)
    v /= np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-12)
    return np.minimum(255.0, np.round(512.0 * v)).astype(np.uint8)


class Corridor:
    """Point cloud + trajectory; images are generated on demand."""

    def __init__(self, num_images: int, num_kpts: int, overlap: int, seed: int,
                 outlier_frac: float = 0.3, noise_px: float = 0.5,
                 desc_noise: float = 0.35, focal: float = 1200.0,
                 confuser_frac: float = 0.1):
        self._kw = dict(num_images=num_images, num_kpts=num_kpts, overlap=overlap, seed=seed,
                        outlier_frac=outlier_frac, noise_px=noise_px, desc_noise=desc_noise,
                        focal=focal, confuser_frac=confuser_frac)
        self.num_images = num_images
        self.num_kpts = num_kpts
        self.seed = seed
        self.outlier_frac = outlier_frac
        self.noise_px = noise_px
        self.desc_noise = desc_noise
        self.focal = focal
        self.confuser_frac = confuser_frac
        self.overlap = overlap
        self.visible = max(8, int(round(num_kpts * (1.0 - outlier_frac))))
        self.step = max(1, self.visible // max(2, overlap))
        self.num_points = self.visible + self.step * num_images
        self.dx = 0.004
        self._blocks = {}

    # Point positions and base descriptors are generated lazily in blocks of
    # 4096 points (seeded per block), so any image of a very long sequence
    # can be produced without materialising the whole corridor.
    _BLOCK = 4096

    def _block(self, b: int):
        blk = self._blocks.get(b)
        if blk is None:
            rng = np.random.default_rng((self.seed, 3, b))
            n = self._BLOCK
            j = np.arange(b * n, (b + 1) * n)
            pts = np.stack([j * self.dx + rng.uniform(-0.5, 0.5, n) * self.dx,
                            rng.uniform(-3.0, 3.0, n), rng.uniform(8.0, 25.0, n)], axis=1)
            # Sparse, heavy-tailed base descriptors (SIFT-like histograms).
            base = rng.gamma(0.5, 1.0, size=(n, 128)).astype(np.float32)
            if len(self._blocks) > 64:
                self._blocks.clear()
            blk = self._blocks[b] = (pts, base)
        return blk

    def _points(self, idx: np.ndarray):
        idx = np.asarray(idx)
        pts = np.empty((len(idx), 3))
        base = np.empty((len(idx), 128), np.float32)
        blocks = idx // self._BLOCK
        for b in np.unique(blocks):
            sel = blocks == b
            p, d = self._block(int(b))
            pts[sel] = p[idx[sel] - b * self._BLOCK]
            base[sel] = d[idx[sel] - b * self._BLOCK]
        return pts, base

    def camera(self, i: int):
        rng = np.random.default_rng((self.seed, 7, i))
        c = np.array([(i * self.step + self.visible / 2) * self.dx,
                      0.2 * np.sin(i / 5.0), -0.5])
        yaw = rng.uniform(-0.03, 0.03)
        pitch = rng.uniform(-0.02, 0.02)
        cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
        Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
        Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
        return Rx @ Ry, c

    def image(self, i: int):
        """(image_id, keypoints N x 6 float32, descriptors N x 128 uint8)."""
        rng = np.random.default_rng((self.seed, 11, i))
        n = self.num_kpts
        nvis = min(self.visible, n)
        idx = np.arange(i * self.step, i * self.step + nvis)
        R, c = self.camera(i)
        P, b = self._points(idx)
        Xc = (P - c) @ R.T
        u = self.focal * Xc[:, 0] / Xc[:, 2] + 960.0 + rng.normal(0, self.noise_px, nvis)
        v = self.focal * Xc[:, 1] / Xc[:, 2] + 540.0 + rng.normal(0, self.noise_px, nvis)
        d_in = b + self.desc_noise * rng.gamma(0.5, 1.0, size=b.shape).astype(np.float32)
        nout = n - nvis
        d_out = rng.gamma(0.5, 1.0, size=(nout, 128)).astype(np.float32)
        # Confusers: outlier keypoints carrying the descriptor of a point that
        # is NOT visible here but is in the next images -> geometrically wrong
        # matches that pass the ratio test (RANSAC outliers).
        ncf = min(nout, int(round(self.confuser_frac * n)))
        if ncf > 0:
            lo = i * self.step + nvis
            hi = min(self.num_points, lo + self.step * max(1, self.overlap))
            if hi > lo:
                pts = rng.integers(lo, hi, size=ncf)
                d_out[:ncf] = self._points(pts)[1] + self.desc_noise * rng.gamma(
                    0.5, 1.0, size=(ncf, 128)).astype(np.float32)
        xy_out = np.stack([rng.uniform(0, 1920, nout), rng.uniform(0, 1080, nout)], axis=1)
        xy = np.concatenate([np.stack([u, v], axis=1), xy_out]).astype(np.float32)
        desc = rootsift_u8(np.concatenate([d_in, d_out]))
        perm = rng.permutation(n)
        kp = np.zeros((n, 6), dtype=np.float32)
        kp[:, 0:2] = xy[perm]
        kp[:, 2] = 1.0
        kp[:, 5] = 1.0
        return i + 1, kp, np.ascontiguousarray(desc[perm])

    def images(self, start: int = 0, stop: int | None = None, workers: int = 1):
        """Images [start, stop); `workers` > 1 generates in forked processes
        (call before any GPU runtime is initialised in this process)."""
        stop = self.num_images if stop is None else min(stop, self.num_images)
        if workers <= 1 or stop - start < 2 * workers:
            return [self.image(i) for i in range(start, stop)]
        import multiprocessing as mp
        global _POOL_CORRIDOR
        _POOL_CORRIDOR = self
        pool = mp.get_context("fork").Pool(workers)
        try:
            out = pool.map(_pool_image, range(start, stop), chunksize=4)
        finally:
            pool.close()  # let the workers exit on their own (no SIGTERM from terminate())
            pool.join()
        return out

    def table_rows_spawned(self, start: int = 0, stop: int | None = None, workers: int = 16,
                           chunk: int = 50):
        """codecs.table_rows of images [start, stop), generated and encoded
        in `workers` spawned processes (safe once the GPU runtime is up in
        this process: nothing is forked from it)."""
        import multiprocessing as mp
        stop = self.num_images if stop is None else min(stop, self.num_images)
        jobs = [(self._kw, a, min(stop, a + chunk)) for a in range(start, stop, chunk)]
        ids, kps, descs = [], [], []
        with mp.get_context("spawn").Pool(workers) as pool:
            for a, b, c in pool.imap(_encoded_chunk, jobs):
                ids += a
                kps += b
                descs += c
        return ids, kps, descs


_POOL_CORRIDOR = None


def _encoded_chunk(job):
    from .codecs import table_rows
    kw, a, b = job
    c = Corridor(**kw)
    return table_rows([c.image(i) for i in range(a, b)])


def _pool_image(i):
    return _POOL_CORRIDOR.image(i)


def random_descriptors(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rootsift_u8(rng.gamma(0.5, 1.0, size=(n, 128)))


def tie_stress_pair(n1: int, n2: int, seed: int):
    """Descriptor pair with duplicate rows, exact ties, zero rows and
    saturated (255) entries: exercises lowest-index tie breaking and the
    best == second ratio-test branch."""
    rng = np.random.default_rng(seed)
    a = random_descriptors(n1, seed)
    b = random_descriptors(n2, seed + 1)
    k = min(n1, n2) // 4
    b[:k] = a[rng.permutation(n1)[:k]]                 # true matches
    b[k:2 * k] = b[:k]                                   # duplicated columns -> ties
    a[n1 // 2: n1 // 2 + k // 2] = a[: k // 2]           # duplicated rows
    a[-3:] = 0                                           # zero rows
    b[-2:] = 0
    a[5, :] = 255                                        # saturated rows
    b[7, :] = 255
    return a, b


def geometry_scene(kind: str, num_matches: int, seed: int, outlier_frac: float = 0.2,
                   noise_px: float = 0.5):
    """Keypoints of two images and a match list whose geometry drives
    TwoViewGeometry::EstimateUncalibrated into a chosen branch (reference
    sequential_matching.cc:98-99 and the post-filter :164-178):

    * "general":     a 3-D scene seen by two cameras -> UNCALIBRATED (3);
    * "planar":      every inlier on one plane (x2 = H x1)
                     -> PLANAR_OR_PANORAMIC (6): H explains > 80 % of the F inliers;
    * "translation": x2 = x1 + t for the inliers, which a 2-D translation
                     explains -> WATERMARK (7) (DetectWatermark; the dummy cameras
                     put every inlier "in the border");
    * "random":      no geometry at all: F and H both find < 15 inliers
                     -> DEGENERATE (1), which the op's post-filter turns into
                     TwoViewGeometry() (config 0);
    * "two_motions": a static 3-D scene (60 % of the matches) and an object
                     moving on its own (the rest before the outliers): two
                     epipolar geometries, so EstimateMultiple (multiple_models)
                     finds both -> MULTIPLE (8); plain Estimate -> UNCALIBRATED.
    * "two_translations": x2 = x1 + t for 76 % of the matches and
                     x2 = x1 + 1.6 t for the rest (one epipolar geometry for
                     both, F = [t]x; H and the watermark's 2-D translation
                     explain only the first set) -> WATERMARK (7), decided by
                     the watermark RANSAC's samples: the first match in
                     index order belongs to the 24 % set, so a RANSAC that
                     sampled only it would find 24 % (< 0.7).
    * "plane_and_depth": a rigid 3-D scene whose first 45 % of points lie on
                     one plane: F explains every inlier and stops within a few
                     dozen trials, H only the plane, so its dynamic trial bound
                     (~500) ends H in the middle of a small batch's second
                     window -> UNCALIBRATED (3).

    Returns (kp1 N x 6, kp2 N x 6, matches M x 2 uint32); keypoint order is
    shuffled so the match indices are not the identity."""
    rng = np.random.default_rng(seed)
    m = num_matches
    x1 = np.stack([rng.uniform(0, 1920, m), rng.uniform(0, 1080, m)], axis=1)
    if kind == "planar":
        H = np.array([[0.92, 0.06, 41.0], [-0.03, 1.04, 18.5], [2.0e-5, -1.5e-5, 1.0]])
        p = np.c_[x1, np.ones(m)] @ H.T
        x2 = p[:, :2] / p[:, 2:3]
    elif kind == "translation":
        x2 = x1 + np.array([37.5, -12.25])
    elif kind == "two_translations":
        t = np.array([37.5, -12.25])
        x2 = x1 + t
        x2[int(round(0.76 * m)):] += 0.6 * t
    elif kind == "random":
        x2 = np.stack([rng.uniform(0, 1920, m), rng.uniform(0, 1080, m)], axis=1)
    elif kind in ("general", "two_motions", "plane_and_depth"):
        X = np.stack([rng.uniform(-4, 4, m), rng.uniform(-2.5, 2.5, m), rng.uniform(6, 20, m)], 1)
        if kind == "plane_and_depth":
            X[:int(round(0.45 * m)), 2] = 10.0
        f = 1200.0

        def proj(R, c, P=None):
            Xc = ((X if P is None else P) - c) @ R.T
            return np.stack([f * Xc[:, 0] / Xc[:, 2] + 960, f * Xc[:, 1] / Xc[:, 2] + 540], 1)
        a = 0.12
        R2 = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        x1 = proj(np.eye(3), np.zeros(3))
        x2 = proj(R2, np.array([1.5, 0.2, 0.3]))
        if kind == "two_motions":  # the last 40 %: an object rotating and sliding on its own
            k = int(round(0.6 * m))
            b = -0.2
            Rb = np.array([[1, 0, 0], [0, np.cos(b), -np.sin(b)], [0, np.sin(b), np.cos(b)]])
            Xo = (X[k:] - np.array([0.0, 0.0, 12.0])) @ Rb.T + np.array([-1.2, 0.8, 12.5])
            x2[k:] = proj(R2, np.array([1.5, 0.2, 0.3]), Xo)
    else:
        raise ValueError(kind)
    x2 = x2 + rng.normal(0, noise_px, x2.shape)
    nout = int(round(outlier_frac * m))
    if nout:
        x2[:nout] = np.stack([rng.uniform(0, 1920, nout), rng.uniform(0, 1080, nout)], axis=1)
    p1 = rng.permutation(m)
    p2 = rng.permutation(m)
    if kind == "two_translations":  # keypoint 0 of image 1 (the first match) in the 24 % set
        j0 = int(np.argmin(p1))
        p1[[j0, m - 1]] = p1[[m - 1, j0]]
    kp1 = np.zeros((m, 6), np.float32)
    kp2 = np.zeros((m, 6), np.float32)
    kp1[p1, :2] = x1
    kp2[p2, :2] = x2
    kp1[:, 2] = kp1[:, 5] = kp2[:, 2] = kp2[:, 5] = 1.0
    matches = np.stack([p1, p2], axis=1).astype(np.uint32)
    matches = matches[np.argsort(matches[:, 0], kind="stable")]  # idx1 ascending, as the matcher
    return kp1, kp2, matches


def descriptors_for_matches(matches: np.ndarray, n1: int, n2: int, seed: int):
    """Descriptor pair whose cross-checked matches are exactly `matches`
    (idx1 ascending, one-to-one): each matched column is a copy of its row's
    RootSIFT descriptor, every other row and column is random.  Lets a
    geometry_scene run through the matcher of the table path."""
    d1 = random_descriptors(n1, seed)
    d2 = random_descriptors(n2, seed + 1)
    d2[matches[:, 1]] = d1[matches[:, 0]]
    return d1, d2


def synthetic_frame(height: int, width: int, seed: int, channels: int = 3,
                    blobs: int | None = None) -> np.ndarray:
    """A deterministic textured frame (H x W x C uint8) for the SIFT extraction
    path: a smooth background, Gaussian blobs of random size, sign and
    position (the DoG detector's natural keypoints), a few oriented bars (so
    orientations and descriptors vary) and mild per-pixel noise; the colour
    channels differ so the grey conversion's channel weights matter."""
    rng = np.random.default_rng(seed)
    h, w = height, width
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.zeros((h, w), np.float32)
    img += 0.3 + 0.15 * np.sin(xx / max(8.0, w / 7.0)) * np.cos(yy / max(8.0, h / 5.0))
    nb = blobs if blobs is not None else max(8, (h * w) // 500)
    for _ in range(nb):
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        s = float(np.exp(rng.uniform(np.log(1.2), np.log(max(2.0, min(h, w) / 30.0)))))
        a = rng.uniform(-0.5, 0.5)
        r = int(4 * s) + 1
        x0, x1 = max(0, int(cx) - r), min(w, int(cx) + r + 1)
        y0, y1 = max(0, int(cy) - r), min(h, int(cy) + r + 1)
        if x0 >= x1 or y0 >= y1:
            continue
        sx, sy = s * rng.uniform(0.6, 1.6), s
        th = rng.uniform(0, np.pi)
        dx, dy = xx[y0:y1, x0:x1] - cx, yy[y0:y1, x0:x1] - cy
        u = np.cos(th) * dx + np.sin(th) * dy
        v = -np.sin(th) * dx + np.cos(th) * dy
        img[y0:y1, x0:x1] += a * np.exp(-0.5 * ((u / sx) ** 2 + (v / sy) ** 2))
    for _ in range(max(2, nb // 20)):  # oriented bars
        cx, cy = rng.uniform(0, w), rng.uniform(0, h)
        th = rng.uniform(0, np.pi)
        ln, wd = rng.uniform(10, max(12.0, min(h, w) / 4)), rng.uniform(1.0, 3.0)
        r = int(ln + wd) + 1
        x0, x1 = max(0, int(cx) - r), min(w, int(cx) + r + 1)
        y0, y1 = max(0, int(cy) - r), min(h, int(cy) + r + 1)
        dx, dy = xx[y0:y1, x0:x1] - cx, yy[y0:y1, x0:x1] - cy
        u = np.cos(th) * dx + np.sin(th) * dy
        v = -np.sin(th) * dx + np.cos(th) * dy
        img[y0:y1, x0:x1] += rng.uniform(-0.3, 0.3) * ((np.abs(u) < ln) & (np.abs(v) < wd))
    img += rng.normal(0, 0.01, img.shape).astype(np.float32)
    base = np.clip(img, 0.0, 1.0) * 255.0
    chans = [np.clip(base * g + o, 0, 255) for g, o in ((1.0, 0.0), (0.9, 12.0), (1.1, -10.0))]
    out = np.stack(chans[:max(1, min(3, channels))], axis=2)
    if channels == 4:
        out = np.concatenate([out, np.full((h, w, 1), 255.0, np.float32)], axis=2)
    return np.rint(out).astype(np.uint8)
