"""Host model of rs_shuffle_wave_body (verify_kernels.hip): RandomSampler's
persistent-vector Shuffle (util/random.h: for i < kmin:
std::swap(sidx[i], sidx[RandomInteger(i, n - 1)])) split in time into chunks
that run on symbols (phase A) and are then applied in order as exit maps
(phase B).  The chunked form must give every trial's sample and the final
vector exactly as the sequential chain, for any targets -- repeated targets
inside a chunk, targets in the head (j < kmin), tiny vectors where nearly
every swap collides."""
import numpy as np
import pytest


def sequential(v, targets, km):
    v = list(v)
    samples = []
    for t in targets:
        for i in range(km):
            j = int(t[i])
            v[i], v[j] = v[j], v[i]
        samples.append(v[:km])
    return samples, v


def chunked(v, targets, km, chunk):
    v = list(v)
    samples = []
    for c0 in range(0, len(targets), chunk):
        # phase A: symbols = positions at the chunk's start
        head = list(range(km))
        table = {}  # touched position -> symbol now there
        sym_samples = []
        for t in targets[c0:c0 + chunk]:
            for i in range(km):
                j = int(t[i])
                if j < km:
                    head[i], head[j] = head[j], head[i]
                else:
                    s = table.get(j, j)
                    table[j] = head[i]
                    head[i] = s
            sym_samples.append(list(head))
        # phase B: samples read the vector at their symbols, then the exit
        # map moves every touched position (all reads before the writes)
        samples += [[v[s] for s in row] for row in sym_samples]
        moves = [(p, v[s]) for p, s in table.items()] + [(i, v[head[i]]) for i in range(km)]
        for p, val in moves:
            v[p] = val
    return samples, v


@pytest.mark.parametrize("km", [4, 7])
@pytest.mark.parametrize("n", [7, 8, 12, 40, 3000])
@pytest.mark.parametrize("chunk", [1, 3, 16])
def test_chunked_shuffle_equals_sequential(km, n, chunk):
    if n < km:
        pytest.skip("fewer matches than the minimal sample")
    rng = np.random.default_rng(n * 31 + km * 7 + chunk)
    trials = 200
    targets = [[int(rng.integers(i, n)) for i in range(km)] for _ in range(trials)]
    v0 = rng.permutation(n).tolist()
    s1, f1 = sequential(v0, targets, km)
    s2, f2 = chunked(v0, targets, km, chunk)
    assert s1 == s2
    assert f1 == f2


def test_chunked_shuffle_repeated_targets():
    """Every swap of a chunk on the same cold position, and head-only swaps."""
    km, n = 7, 20
    targets = [[9] * km for _ in range(20)] + [[i for i in range(km)] for _ in range(5)] + \
              [[km - 1] * km for _ in range(7)]
    v0 = list(range(100, 100 + n))
    for chunk in (1, 2, 5, 16):
        assert chunked(v0, targets, km, chunk) == sequential(v0, targets, km)
