"""Known-answer tests pinning the CPU oracle's two-view geometry
(oracle/oracle.cc: LORANSAC F / H / translation, ComputeNumTrials, the
std::mt19937 + uniform_int_distribution sampler, verify_pair; SURVEY.md §8a
a8-a16).  The reference ships no fixtures for this path (§8c)."""
import math
import struct

import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd.codecs import TVG_HEADER, decode_tvg
from scanner_colmap_amd.synthetic import Corridor


# --- std::mt19937 + libstdc++ uniform_int_distribution<uint32_t> ------------
class MT19937:
    """std::mt19937 (seed via the standard's init_genrand recurrence)."""

    def __init__(self, seed=5489):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            prev = self.mt[i - 1]
            self.mt[i] = (1812433253 * (prev ^ (prev >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __call__(self):
        if self.i >= 624:
            mt = self.mt
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7FFFFFFF)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y


def uniform_u32(g, lo, hi):
    """libstdc++ (GCC >= 11) uniform_int_distribution<uint32_t>::operator()
    for a 32-bit engine: Lemire's nearly-divisionless _S_nd."""
    urange = hi - lo
    if urange == 0xFFFFFFFF:
        return g() + lo
    r = urange + 1
    prod = g() * r
    low = prod & 0xFFFFFFFF
    if low < r:
        threshold = ((1 << 32) - r) % r
        while low < threshold:
            prod = g() * r
            low = prod & 0xFFFFFFFF
    return (prod >> 32) + lo


def test_mt19937_standard_known_answer():
    """C++ standard [rand.predef]: the 10000th output of a default-constructed
    mt19937 is 4123659995."""
    g = MT19937()
    for _ in range(9999):
        g()
    assert g() == 4123659995


def test_uniform_int_distribution_restatement_matches_libstdcxx():
    rng = np.random.default_rng(3)
    hi = rng.integers(0, 2**32, 3000, dtype=np.uint64)
    hi[:500] = rng.integers(0, 20, 500)           # small ranges: RANSAC sample draws
    hi[500:510] = 0xFFFFFFFF
    lo = (rng.random(3000) * hi * 0.3).astype(np.uint64)
    lo[:500] = 0
    lo[500:505] = 0
    got = oracle.std_uniform(1234, lo.astype(np.uint32), hi.astype(np.uint32))
    g = MT19937(1234)
    ref = [uniform_u32(g, int(a), int(b)) for a, b in zip(lo, hi)]
    assert (got == np.array(ref, np.uint32)).all()


# --- ComputeNumTrials --------------------------------------------------------
def num_trials_libm(ni, ns, conf, mult, kmin):
    """COLMAP ComputeNumTrials with std::pow / std::log (glibc via math)."""
    ratio = ni / ns
    nom = 1.0 - conf
    if nom <= 0:
        return 2**64 - 1
    denom = 1.0 - math.pow(ratio, kmin)
    if denom <= 0:
        return 1
    with np.errstate(divide="ignore"):
        v = math.ceil(math.log(nom) / math.log(denom) * mult) if denom < 1 else None
    if v is None:  # log(1) = 0 -> -inf -> static_cast<size_t>(-inf) on x86-64
        return 1 << 63
    return v


def test_num_trials_known_values():
    # 25% inliers over 1e5 samples, 7-pt F: the RANSAC trial cap of SURVEY §8a a10
    assert oracle.num_trials(25000, 100000, 0.999, 3.0, 7) == 339520
    assert oracle.num_trials(100, 100, 0.999, 3.0, 7) == 1
    assert oracle.num_trials(50, 100, 0.999, 3.0, 4) == num_trials_libm(50, 100, 0.999, 3.0, 4)


@pytest.mark.parametrize("kmin", [1, 4, 7, 8])
def test_num_trials_matches_libm_on_grid(kmin):
    """The libm-free restatement (geom_solvers.h num_trials) agrees with the
    std::pow/std::log formula on every (inliers, samples) of the grid, up to
    2^31 (above that only the trial cap max_num_trials <= 2^31 - 1 is used;
    counts near 1e16 differ by an ulp of the double, which cannot matter)."""
    bad = []
    for ns in (15, 16, 50, 97, 100, 500, 1000, 2048, 4096, 8192):
        for ni in range(1, ns + 1, max(1, ns // 300)):
            a = min(oracle.num_trials(ni, ns, 0.999, 3.0, kmin), 2**31)
            b = min(num_trials_libm(ni, ns, 0.999, 3.0, kmin), 2**31)
            if a != b:
                bad.append((ns, ni, a, b))
    assert not bad, bad[:10]


# --- estimators inside LO-RANSAC ----------------------------------------------
def _scene(n, seed, planar=False):
    rng = np.random.default_rng(seed)
    if planar:
        X = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1, 1, n), np.full(n, 10.0)], 1)
    else:
        X = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1, 1, n), rng.uniform(6, 14, n)], 1)
    f = 1000.0
    K = np.array([[f, 0, 960], [0, f, 540], [0, 0, 1.0]])
    a = 0.05
    R = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    t = np.array([-0.6, 0.05, 0.02])
    x1 = (K @ X.T).T
    x1 = x1[:, :2] / x1[:, 2:]
    X2 = X @ R.T + t
    x2 = (K @ X2.T).T
    x2 = x2[:, :2] / x2[:, 2:]
    return x1, x2


def _sampson(F, x1, x2):
    h1 = np.c_[x1, np.ones(len(x1))]
    h2 = np.c_[x2, np.ones(len(x2))]
    Fx1 = h1 @ F.T
    Ftx2 = h2 @ F
    num = np.sum(h2 * Fx1, axis=1) ** 2
    return num / (Fx1[:, 0] ** 2 + Fx1[:, 1] ** 2 + Ftx2[:, 0] ** 2 + Ftx2[:, 1] ** 2)


def test_loransac_fundamental_exact_scene():
    x1, x2 = _scene(200, 1)
    r = oracle.loransac(0, x1, x2, seed=7)
    assert r["success"] and r["num_inliers"] == 200 and r["mask"].all()
    F = r["model"].reshape(3, 3)
    assert np.max(_sampson(F, x1, x2)) < 1e-6
    assert r["num_trials"] >= 30  # min_num_trials


def test_loransac_fundamental_with_outliers():
    x1, x2 = _scene(300, 2)
    rng = np.random.default_rng(5)
    out = rng.choice(300, 90, replace=False)
    x2 = x2.copy()
    x2[out] = rng.uniform([0, 0], [1920, 1080], (90, 2))
    r = oracle.loransac(0, x1, x2, seed=11)
    assert r["success"]
    inl = np.setdiff1d(np.arange(300), out)
    assert r["mask"][inl].all()
    res = _sampson(r["model"].reshape(3, 3), x1, x2)
    assert np.array_equal(r["mask"], res <= 16.0)
    # the reported residual sum is the sum over inliers (tolerance: summation order)
    assert r["residual_sum"] == pytest.approx(res[res <= 16.0].sum(), rel=1e-9, abs=1e-12)


def test_loransac_homography_planar_scene():
    x1, x2 = _scene(150, 3, planar=True)
    r = oracle.loransac(1, x1, x2, seed=3)
    assert r["success"] and r["num_inliers"] == 150
    H = r["model"].reshape(3, 3)
    p = np.c_[x1, np.ones(150)] @ H.T
    assert np.max(np.abs(p[:, :2] / p[:, 2:] - x2)) < 1e-6


def test_loransac_translation():
    rng = np.random.default_rng(9)
    x1 = rng.uniform(0, 1000, (60, 2))
    x2 = x1 + np.array([12.5, -3.25])
    x2[:10] += rng.uniform(50, 100, (10, 2))
    r = oracle.loransac(2, x1, x2, seed=1)
    assert r["success"] and r["num_inliers"] == 50
    assert np.allclose(r["model"][:2], [12.5, -3.25], atol=1e-9)


def test_loransac_deterministic_per_seed():
    x1, x2 = _scene(120, 4)
    x2 = x2 + np.random.default_rng(0).normal(0, 1.0, x2.shape)
    a = oracle.loransac(0, x1, x2, seed=5)
    b = oracle.loransac(0, x1, x2, seed=5)
    assert np.array_equal(a["model"], b["model"]) and a["num_trials"] == b["num_trials"]


# --- verify_pair (TwoViewGeometry::Estimate + post-filter) --------------------
def test_verify_pair_corridor():
    imgs = Corridor(3, 1500, 4, seed=17).images()
    m = oracle.match_pair(imgs[0][2], imgs[1][2])
    blob = oracle.verify_pair(imgs[0][1], imgs[1][1], m, imgs[0][0], imgs[1][0])
    tv = decode_tvg(blob)
    assert tv.config in (3, 6)
    assert len(tv.inlier_matches) >= 15
    assert len(blob) == TVG_HEADER.size + 8 + 8 * len(tv.inlier_matches)
    # inlier matches are a subset of the matches, in order
    mset = {tuple(x) for x in m.tolist()}
    assert all(tuple(x) in mset for x in np.asarray(tv.inlier_matches).tolist())
    assert tv.tri_angle == 0.0
    assert oracle.verify_pair(imgs[0][1], imgs[1][1], m, imgs[0][0], imgs[1][0]) == blob


def test_verify_pair_too_few_matches_is_empty_geometry():
    imgs = Corridor(2, 600, 4, seed=19).images()
    m = oracle.match_pair(imgs[0][2], imgs[1][2])[:14]
    blob = oracle.verify_pair(imgs[0][1], imgs[1][1], m, 1, 2)
    assert len(blob) == 292
    assert struct.unpack_from("<i", blob, 0)[0] == 0
    assert struct.unpack_from("<Q", blob, 284)[0] == 0


# --- the 9 x 9 null-vector solver of the local optimisation (inverse squaring) --
def _pack45(a):
    return np.array([a[p, q] for p in range(9) for q in range(p, 9)])


@pytest.mark.parametrize("seed", range(6))
def test_ata_null_vector_matches_lapack(seed):
    """geom_solvers.h's LO null vector (repeated squaring of (A + delta I)^-1,
    the definition the GPU's lane-per-entry invsq9_null_wave follows bit for
    bit) returns the eigenvector of the smallest eigenvalue of the normal
    matrix to LAPACK accuracy, including near-singular systems (exact data +
    noise)."""
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(400, 9))
    x[:, 8] = 1.0
    x[:, :8] *= rng.uniform(0.05, 3.0, 8)
    if seed % 2:  # one direction almost in the null space
        nvec = rng.normal(size=9)
        nvec /= np.linalg.norm(nvec)
        x -= np.outer(x @ nvec, nvec) * (1.0 - 1e-6)
    a = x.T @ x
    got = oracle.ata_null_vector(_pack45(a))
    w, v = np.linalg.eigh(a)
    ref = v[:, 0]
    assert abs(np.linalg.norm(got) - 1.0) < 1e-12
    assert min(np.abs(got - ref).max(), np.abs(got + ref).max()) < 1e-8 * max(1.0, w[-1] / (w[1] - w[0]) * 1e-8)
    assert np.linalg.norm(a @ got - w[0] * got) <= 1e-9 * w[-1]
