"""The CPU oracle reproduces the committed golden vectors byte for byte
(tests/golden/make_golden.py documents where they come from)."""
import numpy as np
import pytest

from oracle import oracle
from golden_util import MATCH_CASES, VERIFY_CASES, blobs, load, table

G = load()


@pytest.mark.parametrize("case", MATCH_CASES)
def test_golden_matches(case):
    got = oracle.match_pair(G[f"match_{case}_d1"], G[f"match_{case}_d2"])
    ref = G[f"match_{case}_matches"]
    assert got.shape == ref.shape and (got == ref).all()
    if case != "tie_stress":  # every true match there has a duplicate -> rejected
        assert len(ref) > 0


@pytest.mark.parametrize("case", VERIFY_CASES)
def test_golden_verify(case):
    ids = G[f"verify_{case}_ids"]
    got = oracle.verify_pair(G[f"verify_{case}_kp1"], G[f"verify_{case}_kp2"],
                             G[f"verify_{case}_matches"], int(ids[0]), int(ids[1]))
    assert got == G[f"verify_{case}_tvg"].tobytes()


def test_golden_table_rows():
    ids, kps, descs = table(G)
    k = int(G["table_overlap"][0])
    pa, pb = oracle.table_run(ids, kps, descs, k, 0, len(ids))
    assert pa == blobs(G, "table_pairs")
    assert pb == blobs(G, "table_tvgs")


def test_golden_scalars():
    t = int(G["acosf_threshold"][0])
    assert oracle.acosf_normed(t) <= np.float32(0.7) < oracle.acosf_normed(t - 1)
    assert oracle.num_trials(25000, 100000, 0.999, 3.0, 7) == int(G["num_trials_F_cap"][0])
