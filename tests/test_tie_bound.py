"""Host check of the bound behind tie_better (verify_kernels.hip): the inlier
residuals of a model (m values >= 0) summed in index order -- the reference's
InlierSupportMeasurer residual_sum -- and summed in the kernel's any-order
form (per-lane strided partials, then a tree) lie within
E = 2 (m + 2) u T of each other (u = 2^-53, T the any-order sum), so a tie
compare decided from disjoint intervals [T - E, T + E] agrees with the
compare of the ordered sums.  No GPU: the kernel's reduction order is
restated in numpy float64."""
import numpy as np

U = 2.0 ** -53


def seq_sum(x):
    s = 0.0
    for v in x:  # strictly index order, as the reference
        s += float(v)
    return s


def kernel_sum(x, lanes=64, waves=4, unroll=8):
    """The any-order form of tie_better: wave w, lane l takes the points
    i0 + 64 u for i0 = w*64*unroll + l + k*64*unroll*waves (u < unroll) in
    turn, then each wave's 64 partials by the canonical tree, then the waves'
    sums in order."""
    n = len(x)
    part = np.zeros((waves, lanes))
    step = lanes * unroll * waves
    for w in range(waves):
        for l in range(lanes):
            acc = 0.0
            for i0 in range(w * lanes * unroll + l, n, step):
                for u in range(unroll):
                    i = i0 + lanes * u
                    if i < n:
                        acc += float(x[i])
            part[w, l] = acc
    tot = 0.0
    for w in range(waves):
        v = list(part[w])
        width = 32
        while width >= 1:  # lane l += lane l + width
            v = [v[l] + (v[l + width] if l + width < 64 else 0.0) for l in range(64)]
            width //= 2
        tot += v[0]
    return tot


def bound(t, m):
    return 2.0 * (m + 2) * U * t + 1e-300


def test_any_order_sum_within_bound():
    rng = np.random.default_rng(7)
    worst = 0.0
    for trial in range(60):
        m = int(rng.integers(1, 3000))
        kind = trial % 4
        if kind == 0:
            x = rng.uniform(0, 16, m)
        elif kind == 1:  # wide dynamic range
            x = 16.0 * 10.0 ** rng.uniform(-12, 0, m)
        elif kind == 2:  # one large value and many tiny ones
            x = rng.uniform(0, 1e-9, m)
            x[rng.integers(0, m)] = 15.9
        else:  # values one ulp apart, the near-tie regime
            x = np.full(m, 3.0) + rng.integers(0, 4, m) * np.spacing(3.0)
        s, t = seq_sum(x), kernel_sum(x)
        assert abs(s - t) <= bound(t, m), (trial, m, s, t)
        worst = max(worst, abs(s - t) / bound(t, m))
    assert worst < 1.0


def test_disjoint_intervals_decide_as_ordered_sums():
    rng = np.random.default_rng(11)
    decided = 0
    for trial in range(80):
        m = int(rng.integers(20, 1500))
        a = rng.uniform(0, 16, m)
        b = a.copy()
        # perturb a few residuals by a few ulps .. a relative 1e-9
        k = int(rng.integers(1, 5))
        idx = rng.integers(0, m, k)
        b[idx] *= 1.0 + rng.choice([1e-15, 1e-13, 1e-11, 1e-9]) * rng.choice([-1, 1])
        ta, tb = kernel_sum(a), kernel_sum(b)
        ea, eb = bound(ta, m), bound(tb, m)
        better_seq = seq_sum(a) < seq_sum(b)
        if ta + ea < tb - eb:
            assert better_seq
            decided += 1
        elif ta - ea > tb + eb:
            assert not better_seq
            decided += 1
    assert decided > 20  # the bound is tight enough to decide most perturbed pairs
