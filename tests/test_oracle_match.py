"""Known-answer tests pinning the CPU oracle's matcher (oracle/oracle.cc:
compute_sift_distance_matrix / find_best_matches_one_way / cross-check,
SURVEY.md §8a a5-a7) against an independent numpy restatement and
hand-built cases.  The reference ships no tests or fixtures for this path
(SURVEY.md §8c), so these pin the restatement itself."""
import ctypes

import numpy as np
import pytest

from oracle import oracle
from scanner_colmap_amd.synthetic import random_descriptors, tie_stress_pair

_libm = ctypes.CDLL("libm.so.6")
_libm.acosf.restype = ctypes.c_float
_libm.acosf.argtypes = [ctypes.c_float]
F32 = np.float32
K_DIST_NORM = F32(1.0) / (F32(512.0) * F32(512.0))


def acos_normed(d):
    """std::acos(std::min(kDistNorm * d, 1.0f)) in float, glibc acosf."""
    x = min(F32(K_DIST_NORM * F32(d)), F32(1.0))
    return F32(_libm.acosf(float(x)))


def top2_np(dots):
    """FindBestMatchesOneWay scan, vectorised: best = max value
    (lowest index on ties), second = max over the rest including other
    copies of the best value; 0 never becomes best."""
    n1, n2 = dots.shape
    if n2 == 0:
        z = np.zeros(n1, np.int64)
        return z, z, np.full(n1, -1)
    idx = np.argmax(dots, axis=1)  # first occurrence = lowest index
    best = dots[np.arange(n1), idx]
    masked = dots.copy()
    masked[np.arange(n1), idx] = -1
    second = masked.max(axis=1) if n2 > 1 else np.zeros(n1, np.int64)
    second = np.maximum(second, 0)
    idx = np.where(best > 0, idx, -1)
    best = np.where(best > 0, best, 0)
    return best, second, idx


def one_way_np(dots, max_ratio=F32(0.8), max_distance=F32(0.7)):
    best, second, idx = top2_np(dots)
    out = np.full(dots.shape[0], -1)
    for i in range(dots.shape[0]):
        if idx[i] < 0:
            continue
        bn = acos_normed(best[i])
        if bn > max_distance:
            continue
        sn = acos_normed(second[i])
        if bn >= F32(max_ratio * sn):
            continue
        out[i] = idx[i]
    return out


def match_np(d1, d2, cross_check=True):
    dots = d1.astype(np.int64) @ d2.astype(np.int64).T
    m12 = one_way_np(dots)
    if not cross_check:
        return np.array([(i, j) for i, j in enumerate(m12) if j >= 0], np.uint32).reshape(-1, 2)
    m21 = one_way_np(dots.T)
    return np.array([(i, j) for i, j in enumerate(m12) if j >= 0 and m21[j] == i],
                    np.uint32).reshape(-1, 2)


def test_acosf_table_against_libm():
    rng = np.random.default_rng(1)
    for d in list(range(0, 300)) + list(rng.integers(0, 1 << 19, 2000)) + [1 << 18, (1 << 18) + 1]:
        assert np.float32(oracle.acosf_normed(int(d))) == acos_normed(int(d)), d


def test_max_distance_threshold_is_200499():
    """Smallest best-dot value passing max_distance = 0.7f:
    acosf = 0.69999874 at 200,499 vs 0.7000047 at 200,498."""
    assert oracle.acosf_normed(200499) <= F32(0.7)
    assert oracle.acosf_normed(200498) > F32(0.7)


def _vec_with_dot(target):
    """(a, b) u8 descriptors with a.b == target (a = 255 on 4 dims + 1 on one)."""
    q, r = divmod(target, 255)
    assert q <= 4 * 255 and r <= 255
    a = np.zeros(128, np.uint8)
    b = np.zeros(128, np.uint8)
    a[:4] = 255
    a[4] = 1
    b[:4] = [q // 4 + (1 if k < q % 4 else 0) for k in range(4)]
    b[4] = r
    assert int(a.astype(np.int64) @ b.astype(np.int64)) == target
    return a, b


@pytest.mark.parametrize("target,expect", [(200499, True), (200498, False)])
def test_distance_boundary_match(target, expect):
    a, b = _vec_with_dot(target)
    d1 = a[None]
    d2 = np.stack([b, np.zeros(128, np.uint8)])  # second best = 0 -> ratio passes
    m = oracle.match_pair(d1, d2)
    assert (len(m) == 1) == expect
    if expect:
        assert tuple(m[0]) == (0, 0)


def test_ratio_boundary():
    """bn >= 0.8f * sn rejects: find the exact flip point of `second` for a
    fixed best and check the oracle flips there too."""
    best = 240000
    a, b = _vec_with_dot(best)
    lo, hi = 0, best
    bn = acos_normed(best)
    while lo < hi:  # largest s with bn < 0.8f * acos(s) (acos is non-increasing)
        mid = (lo + hi + 1) // 2
        if bn < F32(F32(0.8) * acos_normed(mid)):
            lo = mid
        else:
            hi = mid - 1
    s_pass = lo
    for s, expect in ((s_pass, True), (s_pass + 1, False)):
        _, c = _vec_with_dot(s)
        d2 = np.stack([c, b])  # best at column 1, second at column 0
        m = oracle.match_pair(a[None], d2, opts=_opts(cross_check=0))
        assert (len(m) == 1) == expect, s
        best_, second_, idx_ = oracle.row_top2(a[None], d2)
        assert (best_[0], second_[0], idx_[0]) == (best, s, 1)


def _opts(**kw):
    o = oracle.default_options()
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def test_ties_keep_lowest_index_and_fill_second():
    a = np.zeros((1, 128), np.uint8)
    a[0, :8] = 200
    b = np.zeros((5, 128), np.uint8)
    b[1, :8] = 100
    b[3, :8] = 100  # duplicate of column 1
    best, second, idx = oracle.row_top2(a, b)
    assert (best[0], second[0], idx[0]) == (160000, 160000, 1)
    # best == second -> ratio test rejects
    assert len(oracle.match_pair(a, b)) == 0


def test_zero_rows_never_match():
    d1 = np.zeros((4, 128), np.uint8)
    d2 = random_descriptors(6, 3)
    best, second, idx = oracle.row_top2(d1, d2)
    assert (idx == -1).all() and (best == 0).all()
    assert len(oracle.match_pair(d1, d2)) == 0
    assert len(oracle.match_pair(d2, d1)) == 0


@pytest.mark.parametrize("n1,n2", [(0, 5), (5, 0), (1, 1), (7, 300), (300, 7), (257, 511)])
def test_match_pair_vs_numpy_random(n1, n2):
    d1 = random_descriptors(n1, 10 + n1)
    d2 = random_descriptors(n2, 20 + n2)
    got = oracle.match_pair(d1, d2)
    ref = match_np(d1, d2)
    assert got.shape == ref.shape and (got == ref).all()


def test_match_pair_vs_numpy_near_duplicates():
    """Second image = noisy copies of the first: many real matches."""
    rng = np.random.default_rng(4)
    d1 = random_descriptors(400, 5)
    noise = rng.integers(-3, 4, size=d1.shape)
    d2 = np.clip(d1.astype(np.int64) + noise, 0, 255).astype(np.uint8)[rng.permutation(400)]
    got = oracle.match_pair(d1, d2)
    ref = match_np(d1, d2)
    assert len(ref) > 100
    assert (got == ref).all()


def test_match_pair_vs_numpy_tie_stress():
    d1, d2 = tie_stress_pair(300, 280, 9)
    got = oracle.match_pair(d1, d2)
    assert (got == match_np(d1, d2)).all()
    got = oracle.match_pair(d1, d2, opts=_opts(cross_check=0))
    assert (got == match_np(d1, d2, cross_check=False)).all()


def test_row_top2_vs_numpy_low_entropy():
    """Descriptors over {0, 1, 2}: massive value ties."""
    rng = np.random.default_rng(8)
    d1 = rng.integers(0, 3, size=(64, 128)).astype(np.uint8)
    d2 = rng.integers(0, 3, size=(200, 128)).astype(np.uint8)
    best, second, idx = oracle.row_top2(d1, d2)
    rb, rs, ri = top2_np(d1.astype(np.int64) @ d2.astype(np.int64).T)
    assert (best == rb).all() and (second == rs).all() and (idx == ri).all()


def test_matches_sorted_and_one_to_one():
    d1, d2 = tie_stress_pair(500, 450, 2)
    m = oracle.match_pair(d1, d2)
    assert (np.diff(m[:, 0].astype(np.int64)) > 0).all()
    assert len(np.unique(m[:, 1])) == len(m)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fast_matcher_equals_faithful(seed):
    """oracle.match_pair_fast (exact BLAS dots + the oracle's scans in
    row-major order, the checker of the full-size GPU tests) returns exactly
    the faithful scalar matcher's list: random, tie-stress, corridor pairs and
    every option variant the GPU tests use."""
    from scanner_colmap_amd.synthetic import Corridor, random_descriptors, tie_stress_pair
    cases = [tie_stress_pair(500, 430, seed), (random_descriptors(300, seed), random_descriptors(280, seed + 9))]
    imgs = Corridor(3, 900, 3, seed=seed).images()
    cases += [(imgs[0][2], imgs[1][2]), (imgs[0][2], imgs[0][2])]
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, size=(200, 128), dtype=np.uint8)
    y = rng.integers(0, 256, size=(210, 128), dtype=np.uint8)
    y[:80] = x[:80]
    y[80:120] = x[:40]
    cases.append((x, y))
    for kw in ({}, dict(max_ratio=1.5, max_distance=3.0), dict(cross_check=0), dict(max_ratio=1.0)):
        o = oracle.default_options()
        for k, v in kw.items():
            setattr(o, k, v)
        for a, b in cases:
            ref = oracle.match_pair(a, b, o)
            got = oracle.match_pair_fast(a, b, o)
            assert got.shape == ref.shape and (got == ref).all(), kw


def test_fast_table_run_equals_faithful():
    from scanner_colmap_amd.codecs import table_rows
    from scanner_colmap_amd.synthetic import Corridor
    imgs = Corridor(7, 500, 4, seed=3).images()
    ids, kps, descs = table_rows(imgs)
    assert oracle.table_run_fast(imgs, 4, 0, 7) == oracle.table_run(ids, kps, descs, 4, 0, 7)
    assert oracle.table_run_fast(imgs, 3, 2, 6) == oracle.table_run(ids, kps, descs, 3, 2, 6)
